# GPU tests, then bench.py without the CPU baseline (timed run + kernel replay)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r03_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r03_gpu_tests.log | tail -6
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 700 python -u bench.py --no-cpu > gpurun_out/r03_bench_nocpu.json 2> gpurun_out/r03_bench_nocpu.err
rc=$?; echo "bench rc=$rc"; tail -4 gpurun_out/r03_bench_nocpu.err
python3 -c "
import json;d=json.load(open('gpurun_out/r03_bench_nocpu.json')); k=d['kernels']
print('value', d['value'], 'dp_ms', k['dp_ms'], 'seed_ms', k['seed_ms'], 'resolve_ms', k['resolve_ms'], 'replay', k['replay_reads_per_s'], 'frac', d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
