# rocprofv3 kernel trace + stats of the DP replay (cohort shapes, default config), and the
# lane kernel's development counters (BT2X_DP_PROF=1)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r04d}
timeout -k 10 400 python -u tools/dp_replay.py --slots 65536 --steps 1 "" > gpurun_out/${TAG}_prep.log 2>&1
rc=$?; echo "prep rc=$rc"; grep -E "config|launches" gpurun_out/${TAG}_prep.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o run -- python3 tools/dp_replay.py --slots 65536 --steps 2 "" ${DP_CFGS} > gpurun_out/${TAG}_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; grep -E "config" gpurun_out/${TAG}_kt.log; [ $rc -eq 0 ] || exit $rc
BT2X_DP_PROF=1 timeout -k 10 300 python -u tools/dp_replay.py --slots 65536 --steps 1 "" > gpurun_out/${TAG}_prof.log 2>&1
echo "prof rc=$?"
