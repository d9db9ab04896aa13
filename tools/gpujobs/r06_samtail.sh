#!/bin/bash
# round 6: SAM record tails on the GPU (bt2x_sam_tails): the kernel's test, the GPU e2e
# suite (every DP mode, the reference's SAM), then an interleaved A/B of the timed run
# against host formatting (BT2X_GPU_SAM=0)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06u}
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_e2e.py \
	-k "sam_tails or bt2x_align_vs_reference or md5" > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
[ "${AB:-1}" = 1 ] || exit 0
TAG=${T}_ab CFGS="x BT2X_GPU_SAM=0 x BT2X_GPU_SAM=0" bash tools/gpujobs/r05_hostab.sh
