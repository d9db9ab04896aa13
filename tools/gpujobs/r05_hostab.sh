#!/bin/bash
# round 5: host-side A/B of the timed C3 run (one run each, no legs): the driver's wait
# (BT2X_SPIN_WAIT=2: sleep-poll) and the pool size
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05s}
i=0
for cfg in ${CFGS:-"x" "BT2X_SPIN_WAIT=2" "x --host-threads 15" "BT2X_SPIN_WAIT=2 --host-threads 15"}; do
	i=$((i+1))
	envs=""; args=""
	for w in $cfg; do case $w in *=*) envs="$envs $w";; x) ;; *) args="$args $w";; esac; done
	env $envs timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --runs 1 --no-cpu --no-legs --no-rep-leg --no-replay $args > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err
	rc=$?; [ $rc -eq 0 ] || { echo "cfg [$cfg] rc=$rc"; exit $rc; }
	python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_$i.json')); e=d['end_to_end']
print('cfg [$cfg]', 'value', d['value'], 'host_us', e.get('host_cpu_us_per_read'), 't_wait', e['stats'].get('t_wait'), 't_gather', e['stats'].get('t_gather'), 't_host', e['stats'].get('t_host'))"
done
