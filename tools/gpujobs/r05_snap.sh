#!/bin/bash
# round 5: GPU e2e + dist tests with the lookahead-state adoption, then the timed C3 run
# with it on / off (BT2X_LA_SNAP=0)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05v}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_e2e.py tests/test_dist.py > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1; do
	BT2X_LA_SNAP=$v timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --runs 1 --no-cpu --no-legs --no-rep-leg --no-replay > gpurun_out/${TAG}_snap$v.json 2> gpurun_out/${TAG}_snap$v.err
	rc=$?; [ $rc -eq 0 ] || { echo "snap=$v rc=$rc"; exit $rc; }
	python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_snap$v.json')); e=d['end_to_end']
print('snap $v value', d['value'], 'host_us', e.get('host_cpu_us_per_read'), 'pcie_gb', e.get('pcie_gb'))"
done
