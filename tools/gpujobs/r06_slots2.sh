#!/bin/bash
# round 6: reads in flight (--slots) for the timed C3 run and the repeat-heavy leg,
# interleaved on one box (malloc on huge pages)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06s4}
i=0
for sl in ${SLOTS:-131072 262144 131072 262144}; do
	i=$((i+1))
	timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --runs 1 --no-cpu --no-legs --no-replay \
		--slots $sl > gpurun_out/${T}_$i.json 2> gpurun_out/${T}_$i.err
	rc=$?; [ $rc -eq 0 ] || { echo "slots $sl rc=$rc"; exit $rc; }
	python3 -c "
import json; d=json.load(open('gpurun_out/${T}_$i.json')); e=d['end_to_end']; r=d['configs_other']['C3_rep50']
print('slots $sl', 'C3', d['value'], 'host_us', e.get('host_cpu_us_per_read'), 'rep50', r['value'], r.get('end_to_end',{}).get('host_cpu_us_per_read'))"
done
