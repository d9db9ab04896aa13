#!/bin/bash
# round 5: the read store -- GPU DP parity + e2e + dist, then one timed C3 run (PCIe bytes)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05q}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_e2e.py tests/test_dist.py > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_gpu_tests.log; grep -E "FAILED|Error" gpurun_out/${TAG}_gpu_tests.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 bench.py --steps 20 --warmup 5 --runs ${RUNS:-1} --no-cpu --no-legs --no-rep-leg --no-replay > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"
python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); e=d['end_to_end']
print('value', d['value'], 'pcie_gb', e.get('pcie_gb'), 'host_us', e.get('host_cpu_us_per_read'), 'gpu', e.get('gpu'))"
exit $rc
