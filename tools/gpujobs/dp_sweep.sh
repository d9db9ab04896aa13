# DP replay only (no tests): configurations in DP_CFGS at cohort and whole-file shapes
mkdir -p gpurun_out
for s in 65536 1048576; do
timeout -k 10 400 python -u tools/dp_replay.py --slots $s "" ${DP_CFGS} > gpurun_out/dp_sweep_$s.log 2>&1
rc=$?; echo "slots $s rc=$rc"; grep -E "config|launches|Error|error" gpurun_out/dp_sweep_$s.log | tail -9
[ $rc -eq 0 ] || exit $rc
done
