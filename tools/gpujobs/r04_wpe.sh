# u8 fused fill at 3 vs 2 waves/SIMD (BT2X_DP_WPE=2: no VGPR spills): DP replay at cohort
# shapes, then the DP parity tests under the 2-wave variant
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python -u tools/dp_replay.py --slots 131072 "" BT2X_DP_WPE=2 "" BT2X_DP_WPE=2 > gpurun_out/r04cc_wpe_131072.log 2>&1
rc=$?; echo "replay rc=$rc"; grep -E "config|launches|Error|error" gpurun_out/r04cc_wpe_131072.log | tail -12
[ $rc -eq 0 ] || exit $rc
BT2X_DP_WPE=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_e2e.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04cc_wpe_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04cc_wpe_tests.log
exit $rc
