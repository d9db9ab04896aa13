#!/bin/bash
# round-6 final C: the same passes over the bench with its legs (C2: the i16 fill; C5; the
# repeat-heavy leg); tools/pmc_traffic.py --segment 1 / 2 (run where the passes' outputs are
# gathered) picks the C2 / rep50 replays.  PASSES selects passes (default all).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/legs
B="bench.py --no-cpu --no-replay-whole --runs 1"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
PASSES=${PASSES:-"kt fetch write sq"}
for ps in $PASSES; do
	case $ps in
	kt) timeout -k 10 560 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/legs/prof_kt -o run -- python3 $B > gpurun_out/legs/prof_kt.log 2>&1 ;;
	fetch) timeout -k 10 560 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/legs/prof_fetch -o run -- python3 $B > gpurun_out/legs/prof_fetch.log 2>&1 ;;
	write) timeout -k 10 560 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/legs/prof_write -o run -- python3 $B > gpurun_out/legs/prof_write.log 2>&1 ;;
	sq) timeout -k 10 560 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d gpurun_out/legs/prof_sq -o run -- python3 $B > gpurun_out/legs/prof_sq.log 2>&1 ;;
	esac
	rc=$?; echo "pass $ps rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
