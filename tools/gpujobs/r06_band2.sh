#!/bin/bash
# round 6: banded layout in the hand-over pass (dp_wave_kernel<2, *, true>) too: DP parity
# (edge shapes, goldens, at-scale set; e2e wave modes), then the replay at cohort shapes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06n}
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
	-k "edge_shapes or production_kernel or at_scale" > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_e2e.py \
	-k "wave or default or handover" > gpurun_out/${T}_e2e.log 2>&1
rc=$?; echo "e2e rc=$rc"; tail -2 gpurun_out/${T}_e2e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o kt -- \
	python3 tools/dp_replay.py --slots 65536 --steps 3 "" BT2X_DP_WAVE_BAND=0 "" > gpurun_out/${T}_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; grep -E "^config" gpurun_out/${T}_kt.log; exit $rc
