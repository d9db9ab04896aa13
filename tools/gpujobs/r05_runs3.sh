#!/bin/bash
# three timed runs of the C3 bench, nothing else (run-to-run spread after the per-run fresh SAM file)
T=${T:-r05bb}; cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python3 bench.py --steps 20 --warmup 5 --runs 3 --no-cpu --no-legs --no-rep-leg --no-replay > gpurun_out/${T}.json 2> gpurun_out/${T}.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json; d=json.load(open('gpurun_out/${T}.json'))
print('value', d['value']); [print(r) for r in d['end_to_end']['runs']]"
