#!/bin/bash
# round 6: the full -m gpu suite, smoke(), then the driver's bench command (N=1)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06z}
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${T}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > gpurun_out/${T}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${T}_smoke.log; [ $rc -eq 0 ] || exit $rc
[ "${BENCH:-1}" = 1 ] || exit 0
timeout -k 10 650 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.load(open('gpurun_out/${T}_bench.json'))
print('value', d['value'], [r['value'] for r in d['end_to_end']['runs']], 'host_us', d['end_to_end']['host_cpu_us_per_read'], 'cpu', d['cpu_baseline']['value'], 'parity', d['parity']['records_differ'], 'frac', d['roofline']['frac'])"
exit $rc
