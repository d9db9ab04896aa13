#!/bin/bash
# round 5: GPU DP parity + e2e + dist with the current walk, then the walk A/B replay
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05l}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_e2e.py tests/test_dist.py > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_gpu_tests.log; grep -E "FAILED|Error" gpurun_out/${TAG}_gpu_tests.log | head -5
[ $rc -eq 0 ] || exit $rc
TAG=$TAG VARIANTS="${VARIANTS:-A main}" bash tools/gpujobs/r05_walkab.sh
