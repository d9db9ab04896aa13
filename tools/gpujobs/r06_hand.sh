#!/bin/bash
# round 6: the wave kernel handing problems of many candidates to the wave-parallel walk
# (BT2X_DP_WAVE_HAND): DP parity, then a replay sweep at cohort shapes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06m}
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py \
	-k "edge_shapes or production_kernel or at_scale" > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/dp_replay.py --slots 65536 --steps 3 "" BT2X_DP_WAVE_HAND=0 BT2X_DP_WAVE_HAND=4 \
	BT2X_DP_WAVE_HAND=8 BT2X_DP_WAVE_HAND=32 "" > gpurun_out/${T}_replay.log 2>&1
rc=$?; echo "replay rc=$rc"; grep -E "^config" gpurun_out/${T}_replay.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o kt -- \
	python3 tools/dp_replay.py --slots 65536 --steps 2 "" > gpurun_out/${T}_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; exit $rc
