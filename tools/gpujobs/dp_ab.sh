# DP replay A/B: ablations and the wave-kernel threshold at cohort and whole-file shapes
mkdir -p gpurun_out
for s in 65536 1048576; do
timeout -k 10 400 python -u tools/dp_replay.py --slots $s "" BT2X_DP_ABLATE=2 BT2X_DP_ABLATE=1 \
  BT2X_DP_WAVE_MAX=65536 BT2X_DP_WAVE_MAX=131072 BT2X_DP_WAVE_MAX=262144 BT2X_DP_WAVE_MAX=16384 \
  > gpurun_out/r03_dp_ab_$s.log 2>&1
rc=$?; echo "slots $s rc=$rc"; grep -E "config|launches|Error|error" gpurun_out/r03_dp_ab_$s.log | tail -9
[ $rc -eq 0 ] || exit $rc
done
