#!/bin/bash
# round 6: per-launch development counters of the DP replay (BT2X_DP_PROF=1): problems
# handed to the wave kernel's hand-over pass per launch
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06o}
BT2X_DP_PROF=1 timeout -k 10 300 python3 tools/dp_replay.py --slots 65536 --steps 1 "" > gpurun_out/${T}_prof.log 2>&1
rc=$?; echo "rc=$rc"; grep -c BT2X_DP_PROF gpurun_out/${T}_prof.log; exit $rc
