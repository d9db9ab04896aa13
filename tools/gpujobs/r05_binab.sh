#!/bin/bash
# round 5: interleaved A/B of two bt2x-align builds on the timed C3 run (one run each, twice)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05bin}
i=0
for b in "$BINA" "$BINB" "$BINA" "$BINB"; do
	i=$((i+1))
	timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --runs 1 --no-cpu --no-legs --no-rep-leg --no-replay \
	  --aligner $GRAFT_REPO_ROOT/$b > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
	rc=$?; [ $rc -eq 0 ] || { echo "[$b] rc=$rc"; exit $rc; }
	python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_$i.json')); e=d['end_to_end']
print('[$b] value', d['value'], 'host_us', e.get('host_cpu_us_per_read'))"
done
