#!/bin/bash
# round 5: the two-lanes-per-problem DP fill (dp_duo_kernel): DP parity + e2e + dist GPU
# tests, then a DP replay at the timed run's cohort shapes, duo vs the one-lane fill
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05b}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_e2e.py tests/test_dist.py > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/dp_replay.py --slots 65536 "" BT2X_DP_DUO=0 ${DP_CFGS} > gpurun_out/${TAG}_dpreplay.log 2>&1
rc=$?; echo "replay rc=$rc"; grep -E "config|DP |ms|Error|error" gpurun_out/${TAG}_dpreplay.log | tail -20
exit $rc
