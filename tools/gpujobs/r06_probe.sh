#!/bin/bash
# round 6: the seed-count check's GPU test, then the DP fill/duo split probe at the timed
# run's cohort shapes (fill only, walk only, both)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06a}
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_round.py tests/test_abi.py > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/dp_replay.py --slots 65536 --steps 3 "" BT2X_DP_DUO=0 BT2X_DP_DUO=1 \
	BT2X_DP_DUO=0,BT2X_DP_ABLATE=1 BT2X_DP_DUO=1,BT2X_DP_ABLATE=1 BT2X_DP_DUO=0,BT2X_DP_ABLATE=2 BT2X_DP_DUO=1,BT2X_DP_ABLATE=2 \
	> gpurun_out/${T}_duo_probe.log 2>&1
rc=$?; echo "replay rc=$rc"; grep -E "^config|^#" gpurun_out/${T}_duo_probe.log; exit $rc
