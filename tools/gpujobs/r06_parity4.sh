#!/bin/bash
# round 6: more C3 parity runs (the differing records are listed when any)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06p4}
for i in 1 2 3; do
	timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 --runs 1 --no-legs --no-rep-leg --no-replay \
		> gpurun_out/${T}_$i.json 2> gpurun_out/${T}_$i.err
	rc=$?; echo "run $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
	python3 -c "
import json; d=json.load(open('gpurun_out/${T}_$i.json')); print(d['value'], json.dumps(d['parity'])[:3000], d['cpu_baseline'].get('reference_runs_differ'), d['cpu_baseline'].get('reference_runs_examples'))"
done
