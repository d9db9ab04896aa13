# rocprofv3 kernel trace of the DP replay at cohort shapes (per-kernel durations)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dprof -o run -- python3 tools/dp_replay.py --slots 65536 --steps 2 "" > gpurun_out/dprof.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/dprof.log; find gpurun_out/dprof -name "*kernel_stats.csv" | head -3
