#!/bin/bash
# round 6: grouped candidate ordering (order_candidates): DP parity (edge shapes with the
# debug kernels' candidate lists, goldens, at-scale set), then the replay at cohort shapes
# and its fill-only ablation, with kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06r}
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
	-k "edge_shapes or production_kernel or at_scale or golden" > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o kt -- \
	python3 tools/dp_replay.py --slots 65536 --steps 3 "" BT2X_DP_ABLATE=1 "" > gpurun_out/${T}_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; grep -E "^config" gpurun_out/${T}_kt.log; exit $rc
