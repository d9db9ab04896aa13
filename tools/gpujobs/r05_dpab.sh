#!/bin/bash
# DP replay A/B at the timed run's cohort shapes (--slots 65536): configs from $DP_CFGS
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05c}
timeout -k 10 900 python -u tools/dp_replay.py --slots ${SLOTS:-65536} --steps ${STEPS:-3} ${DP_CFGS} > gpurun_out/${TAG}_dpreplay.log 2>&1
rc=$?; echo "replay rc=$rc"; grep -E "^config|Error|error" gpurun_out/${TAG}_dpreplay.log | tail -20
exit $rc
