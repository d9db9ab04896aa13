# DP lane-kernel time split (BT2X_DP_PROF=1: fill / walk cycles, walk wave-steps per launch)
mkdir -p gpurun_out
for s in 65536; do
BT2X_DP_PROF=1 timeout -k 10 400 python -u tools/dp_replay.py --slots $s --steps 1 "" > gpurun_out/dp_prof_$s.log 2>&1
rc=$?; echo "slots $s rc=$rc"; grep -E "config|launches|Error|error" gpurun_out/dp_prof_$s.log | tail -3
[ $rc -eq 0 ] || exit $rc
done
