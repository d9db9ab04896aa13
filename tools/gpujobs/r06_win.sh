#!/bin/bash
# round 6: the DP fill's LDS-DMA window ring -- DP parity, then the cohort-shape replay
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06h}
timeout -k 10 420 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py \
	-k "edge_shapes or production_kernel or at_scale or exact_best or read_store or golden" > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/dp_replay.py --slots 65536 --steps 3 "" BT2X_DP_ABLATE=1 BT2X_DP_DUO=0 BT2X_DP_SPLIT=1 \
	> gpurun_out/${T}_replay.log 2>&1
rc=$?; echo "replay rc=$rc"; grep -E "^config|^#" gpurun_out/${T}_replay.log; exit $rc
