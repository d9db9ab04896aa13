#!/bin/bash
# round 5: GPU e2e + dist tests on the current host driver, then the DP lookahead A/B
# (bt2x-align --lookahead: problems posed per DP request) on the timed C3 run
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05u}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_e2e.py tests/test_dist.py tests/test_round.py > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for la in ${LAS:-8 4 6 12}; do
	timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --runs 1 --no-cpu --no-legs --no-rep-leg --no-replay --align-extra=--lookahead,$la > gpurun_out/${TAG}_la$la.json 2> gpurun_out/${TAG}_la$la.err
	rc=$?; [ $rc -eq 0 ] || { echo "la=$la rc=$rc"; exit $rc; }
	python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_la$la.json')); e=d['end_to_end']; s=e['stats']
print('lookahead $la value', d['value'], 'host_us', e.get('host_cpu_us_per_read'), 'dps', s.get('dps'), 'dps_used', s.get('dps_used'), 'dp_launches', s.get('dp_launches'), 'k_dp', e['gpu'].get('k_dp'))"
done
