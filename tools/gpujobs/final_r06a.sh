#!/bin/bash
# round-6 final A: rocprofv3 summaries of the C3 bench (no legs): kernel trace + stats, then
# FETCH_SIZE, WRITE_SIZE and the SQ counters, each in a pass of its own; tools/pmc_traffic.py
# --replays 4 (1 counter step + 3 timed replay steps) turns them into profiles/r06_*.
# PASSES selects passes (default all: "kt fetch write sq summ"), for calls within gpurun's limit.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
B="bench.py --no-cpu --no-legs --no-rep-leg --no-replay-whole --runs 1"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
PASSES=${PASSES:-"kt fetch write sq summ"}
for ps in $PASSES; do
	case $ps in
	kt) timeout -k 10 550 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o run -- python3 $B > gpurun_out/prof_kt.log 2>&1 ;;
	fetch) timeout -k 10 550 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_fetch -o run -- python3 $B > gpurun_out/prof_fetch.log 2>&1 ;;
	write) timeout -k 10 550 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_write -o run -- python3 $B > gpurun_out/prof_write.log 2>&1 ;;
	sq) timeout -k 10 550 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d gpurun_out/prof_sq -o run -- python3 $B > gpurun_out/prof_sq.log 2>&1 ;;
	summ)
		KEY=$(python3 -c "
import json
for ln in open('gpurun_out/prof_kt.log'):
    if ln.startswith('{'): d = json.loads(ln)
print(d['config']['key'])")
		python3 tools/pmc_traffic.py --src gpurun_out --tag r06 --replays 4 --workload "$KEY" --cmd "python3 $B" --out gpurun_out/prof_summ > gpurun_out/prof_summ_a.log 2>&1 ;;
	esac
	rc=$?; echo "pass $ps rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
