#!/bin/bash
# round 5: interleaved host A/B of the timed C3 run and the repeat-heavy leg (one run per setting): ENVA vs ENVB, twice
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05w}
i=0
for e in "$ENVA" "$ENVB" "$ENVA" "$ENVB"; do
	i=$((i+1))
	env $e timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --runs 1 --no-cpu --no-legs --no-replay > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
	rc=$?; [ $rc -eq 0 ] || { echo "[$e] rc=$rc"; exit $rc; }
	python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_$i.json')); e=d['end_to_end']
print('[$e] value', d['value'], 'host_us', e.get('host_cpu_us_per_read'), 'rep50', d.get('configs_other',{}).get('C3_rep50',{}).get('value'))"
done
