# DP walk change: GPU parity tests, then bench (no CPU baseline) at the timed run's cohort
# shapes and with whole-file launches
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r03d_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r03d_gpu_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.err
rc=$?; echo "bench rc=$rc"; tail -4 gpurun_out/r03d_bench.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu --replay-slots 1048576 > gpurun_out/r03d_bench_whole.json 2> gpurun_out/r03d_bench_whole.err
rc=$?; echo "bench whole rc=$rc"; tail -3 gpurun_out/r03d_bench_whole.err; exit $rc
