#!/bin/bash
# round 5: interleaved sweep of bench arguments on the timed C3 run: ARGLIST ("a|b|c"), twice over
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05sw}
IFS='|' read -r -a L <<< "$ARGLIST"
i=0
for pass in 1 2; do
	for e in "${L[@]}"; do
		i=$((i+1))
		timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --runs 1 --no-cpu --no-legs --no-rep-leg --no-replay $e > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
		rc=$?; [ $rc -eq 0 ] || { echo "[$e] rc=$rc"; exit $rc; }
		python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_$i.json')); e=d['end_to_end']
print('[$e] value', d['value'], 'host_us', e.get('host_cpu_us_per_read'))"
	done
done
