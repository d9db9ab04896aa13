#!/bin/bash
# round 6: is the unrolled DP fill instruction-fetch bound?  Instruction-cache counters of the
# fill (no walks: BT2X_DP_ABLATE=1) for the one-lane fill and the two-lane duo fill at the
# timed run's cohort shapes (tools/dp_replay.py), each counter pass its own run
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06b}
(timeout -s KILL 60 rocprofv3 -L > gpurun_out/${T}_counters_list.txt 2>&1 || true)
# the recording (cached under the workdir) first, without the profiler
timeout -k 10 300 python -u tools/dp_replay.py --slots 65536 --steps 1 BT2X_DP_DUO=0,BT2X_DP_ABLATE=1 > gpurun_out/${T}_rec.log 2>&1
rc=$?; echo "record rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for pmc in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVES SQ_INSTS_VALU" "SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY" "SQ_IFETCH SQ_INSTS_SALU SQ_WAIT_ANY SQ_BUSY_CYCLES"; do
	i=$((i+1))
	timeout -s KILL 240 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d gpurun_out/${T}_ic$i -o run -- \
		python3 -u tools/dp_replay.py --slots 65536 --steps 1 BT2X_DP_DUO=0,BT2X_DP_ABLATE=1 BT2X_DP_DUO=1,BT2X_DP_ABLATE=1 \
		> gpurun_out/${T}_ic$i.log 2>&1
	rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
ls -R gpurun_out/${T}_ic1 | head
