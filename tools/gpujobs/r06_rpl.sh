#!/bin/bash
# round 6: the wave kernel with rows-per-lane selection (3 rows a lane at 150 bp) and the
# banded traceback layout: DP parity (edge shapes, goldens, at-scale set, e2e wave modes),
# then the replay at cohort shapes against whole rectangles, then kernel stats of both
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06k}
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py \
	-k "edge_shapes or production_kernel or at_scale or read_store" > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_e2e.py \
	-k "wave or default" > gpurun_out/${T}_e2e.log 2>&1
rc=$?; echo "e2e rc=$rc"; tail -2 gpurun_out/${T}_e2e.log; [ $rc -eq 0 ] || exit $rc
for v in band full; do
	e=""; [ $v = full ] && e="BT2X_DP_WAVE_BAND=0"
	timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt_$v -o kt -- \
		python3 tools/dp_replay.py --slots 65536 --steps 3 "$e" > gpurun_out/${T}_kt_$v.log 2>&1
	rc=$?; echo "$v rc=$rc"; grep -E "^config" gpurun_out/${T}_kt_$v.log; [ $rc -eq 0 ] || exit $rc
done
