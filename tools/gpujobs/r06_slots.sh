#!/bin/bash
# round 6: reads in flight (--slots) with malloc on huge pages: the timed C3 run, interleaved
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06s3}
i=0
for sl in ${SLOTS:-262144 131072 262144 131072}; do
	i=$((i+1))
	timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --runs 1 --no-cpu --no-legs --no-rep-leg --no-replay \
		--slots $sl > gpurun_out/${T}_$i.json 2> gpurun_out/${T}_$i.err
	rc=$?; [ $rc -eq 0 ] || { echo "slots $sl rc=$rc"; exit $rc; }
	python3 -c "
import json; d=json.load(open('gpurun_out/${T}_$i.json')); e=d['end_to_end']
print('slots $sl', 'value', d['value'], 'host_us', e.get('host_cpu_us_per_read'), 't_wait', e['stats'].get('t_wait'), 'rss', e.get('peak_rss_mib'))"
done
