# one DP-kernel iteration: GPU parity tests, then the DP replay (with BT2X_DP_PROF lines) at
# cohort and whole-file shapes
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ \
  > gpurun_out/dp_iter_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/dp_iter_tests.log
[ $rc -eq 0 ] || exit $rc
for s in 65536 1048576; do
timeout -k 10 400 python -u tools/dp_replay.py --slots $s "" ${DP_CFGS} > gpurun_out/dp_iter_$s.log 2>&1
rc=$?; echo "slots $s rc=$rc"; grep -E "config|launches|Error|error" gpurun_out/dp_iter_$s.log | tail -9
[ $rc -eq 0 ] || exit $rc
done
BT2X_DP_PROF=1 timeout -k 10 400 python -u tools/dp_replay.py --slots 65536 --steps 1 "" > gpurun_out/dp_iter_prof.log 2>&1
echo "prof rc=$?"
