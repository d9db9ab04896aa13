#!/bin/bash
# DP replay with BT2X_DP_PROF=1 (per-wave phase cycles of the lane kernels)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05g}
BT2X_DP_PROF=1 timeout -k 10 900 python -u tools/dp_replay.py --slots ${SLOTS:-65536} --steps 1 ${DP_CFGS} > gpurun_out/${TAG}_dpprof.log 2>&1
rc=$?; echo "replay rc=$rc"; grep -E "^config|Error|error" gpurun_out/${TAG}_dpprof.log | tail -20
exit $rc
