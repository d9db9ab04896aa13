#!/bin/bash
# round 6: the small-launch wave kernel's walk on every lane (BT2X_DP_PARWALK=2) against
# lane 0's, per launch (kernel traces of the DP replay at cohort shapes)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06l}
for v in par2 def; do
	e=""; [ $v = par2 ] && e="BT2X_DP_PARWALK=2"
	timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt_$v -o kt -- \
		python3 tools/dp_replay.py --slots 65536 --steps 2 "$e" > gpurun_out/${T}_kt_$v.log 2>&1
	rc=$?; echo "$v rc=$rc"; grep -E "^config" gpurun_out/${T}_kt_$v.log; [ $rc -eq 0 ] || exit $rc
done
