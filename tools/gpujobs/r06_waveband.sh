#!/bin/bash
# round 6: the banded traceback layout of the small-launch wave kernel (dp_wave_kernel<0,
# *, true>): DP parity first, then the DP replay at the timed run's cohort shapes against
# whole rectangles in LDS (BT2X_DP_WAVE_BAND=0), then the replay's kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06i}
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py \
	-k "edge_shapes or production_kernel or at_scale or read_store" > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/dp_replay.py --slots 65536 --steps 3 "" BT2X_DP_WAVE_BAND=0 "" BT2X_DP_WAVE_BAND=0 \
	> gpurun_out/${T}_replay.log 2>&1
rc=$?; echo "replay rc=$rc"; grep -E "^config|^#" gpurun_out/${T}_replay.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_kt -o kt -- python3 tools/dp_replay.py --slots 65536 --steps 1 "" \
	> gpurun_out/${T}_kt.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
