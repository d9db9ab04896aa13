#!/bin/bash
# round-6 final C: the same passes over the bench with its legs (C2: the i16 fill; C5; the
# repeat-heavy leg); tools/pmc_traffic.py --segment 1 / 2 picks the C2 / rep50 replays
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/legs
B="bench.py --no-cpu --no-replay-whole --runs 1"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/legs/prof_kt -o run -- python3 $B > gpurun_out/legs/prof_kt.log 2>&1 && \
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/legs/prof_fetch -o run -- python3 $B > gpurun_out/legs/prof_fetch.log 2>&1 && \
timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/legs/prof_write -o run -- python3 $B > gpurun_out/legs/prof_write.log 2>&1 && \
timeout -k 10 900 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d gpurun_out/legs/prof_sq -o run -- python3 $B > gpurun_out/legs/prof_sq.log 2>&1
rc=$?; echo "profile C rc=$rc"; tail -c 400 gpurun_out/legs/prof_kt.log; [ $rc -eq 0 ] || exit $rc
for seg in 1 2; do
	KEY=$(python3 -c "
import json
for ln in open('gpurun_out/legs/prof_kt.log'):
    if ln.startswith('{'): d = json.loads(ln)
print(d['configs_other']['C2' if $seg == 1 else 'C3_rep50']['workload_key'])")
	TG=$([ $seg = 1 ] && echo r06_c2 || echo r06_rep50)
	python3 tools/pmc_traffic.py --src gpurun_out/legs --tag $TG --replays 4 --segment $seg --workload "$KEY" --cmd "python3 $B" --out gpurun_out/prof_summ > gpurun_out/prof_summ_$TG.log 2>&1
	rc=$?; echo "summary $TG rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
rm -rf gpurun_out/legs/prof_fetch gpurun_out/legs/prof_write gpurun_out/legs/prof_sq; exit 0
