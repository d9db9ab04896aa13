#!/bin/bash
# round 6: run-to-run spread of the timed C3 run (3 runs per bench, each run's rusage), with
# and without malloc on huge pages
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06v2}
i=0
for cfg in x BT2X_MALLOC_THP=0 x; do
	i=$((i+1)); envs=""; [ $cfg = x ] || envs=$cfg
	env $envs timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --runs 3 --no-cpu --no-legs --no-rep-leg --no-replay \
		> gpurun_out/${T}_$i.json 2> gpurun_out/${T}_$i.err
	rc=$?; [ $rc -eq 0 ] || { echo "cfg [$cfg] rc=$rc"; exit $rc; }
	python3 -c "
import json; d=json.load(open('gpurun_out/${T}_$i.json'))
print('cfg [$cfg]', d['value'], [(r['value'], r.get('rusage',{}).get('user'), r.get('rusage',{}).get('sys'), r.get('rusage',{}).get('minflt')) for r in d['end_to_end']['runs']])"
done
