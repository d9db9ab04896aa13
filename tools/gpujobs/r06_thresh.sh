#!/bin/bash
# round 6: launch-size thresholds of the DP kernels at cohort shapes after the wave-kernel and
# candidate-order changes: one wave per problem up to BT2X_DP_WAVE_MAX, the duo fill up to
# BT2X_DP_DUO_MAX
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06t2}
timeout -k 10 600 python -u tools/dp_replay.py --slots 65536 --steps 3 "" BT2X_DP_WAVE_MAX=16384 BT2X_DP_WAVE_MAX=49152 \
	BT2X_DP_WAVE_MAX=65536 BT2X_DP_DUO_MAX=32768 BT2X_DP_DUO_MAX=98304 BT2X_DP_DUO_MAX=131072 "" > gpurun_out/${T}_replay.log 2>&1
rc=$?; echo "replay rc=$rc"; grep -E "^config|^#" gpurun_out/${T}_replay.log; exit $rc
