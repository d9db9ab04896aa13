#!/bin/bash
# round 6: per-launch DP kernel durations at the timed run's cohort shapes, split fill vs
# one-lane fill (rocprofv3 kernel trace of tools/dp_replay.py, fill only and whole DP)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06d}
timeout -k 10 300 python -u tools/dp_replay.py --slots 65536 --steps 1 BT2X_DP_ABLATE=1 > gpurun_out/${T}_rec.log 2>&1
rc=$?; echo "record rc=$rc"; [ $rc -eq 0 ] || exit $rc
for cfg in BT2X_DP_ABLATE=1 BT2X_DP_SPLIT=0,BT2X_DP_DUO=0,BT2X_DP_ABLATE=1 "" BT2X_DP_SPLIT=0,BT2X_DP_DUO=0; do
	n=$(echo "$cfg" | tr ',=' '__')
	timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_kt_${n:-default} -o run -- \
		python3 -u tools/dp_replay.py --slots 65536 --steps 1 "$cfg" > gpurun_out/${T}_kt_${n:-default}.log 2>&1
	rc=$?; echo "trace [$cfg] rc=$rc"; [ $rc -eq 0 ] || exit $rc
	grep -E "^config" gpurun_out/${T}_kt_${n:-default}.log
done
