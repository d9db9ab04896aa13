#!/bin/bash
# round 6: the C2 leg (i16) with larger launches through the wave kernel
# (BT2X_DP_WAVE_MAX), against the default; C3 shrunk to 1 M reads (its numbers unused)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06v}
i=0
for cfg in x BT2X_DP_WAVE_MAX=131072 x BT2X_DP_WAVE_MAX=65536; do
	i=$((i+1)); envs=""; [ $cfg = x ] || envs=$cfg
	env $envs timeout -k 10 500 python3 bench.py --reads 1000000 --steps 2 --warmup 1 --runs 1 --no-cpu --no-rep-leg \
		--no-replay-whole > gpurun_out/${T}_$i.json 2> gpurun_out/${T}_$i.err
	rc=$?; [ $rc -eq 0 ] || { echo "cfg [$cfg] rc=$rc"; exit $rc; }
	python3 -c "
import json; d=json.load(open('gpurun_out/${T}_$i.json')); c=d['configs_other']['C2']
print('cfg [$cfg]', 'C2', c['value'], 'roof_i16', (c.get('roofline_i16') or {}).get('frac'), 'dp_ms', c.get('kernels',{}).get('dp_ms'), 'parity', c['parity']['records_differ'] if isinstance(c.get('parity'),dict) else c.get('parity'))"
done
