#!/bin/bash
# round 6: kernel stats of the DP replay at cohort shapes, banded wave-kernel layout vs
# whole rectangles (BT2X_DP_WAVE_BAND=0)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06j}
for v in band full; do
	e=""; [ $v = full ] && e="BT2X_DP_WAVE_BAND=0"
	timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt_$v -o kt -- \
		python3 tools/dp_replay.py --slots 65536 --steps 2 "$e" > gpurun_out/${T}_kt_$v.log 2>&1
	rc=$?; echo "$v rc=$rc"; grep -E "^config" gpurun_out/${T}_kt_$v.log; [ $rc -eq 0 ] || exit $rc
done
