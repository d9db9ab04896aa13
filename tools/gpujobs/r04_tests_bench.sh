# round 4: the GPU test suite, then bench.py exactly as the driver runs it
# (--gpus 1 --steps 20 --warmup 5); stops after a GPU fault/timeout
mkdir -p gpurun_out
TAG=${TAG:-r04}
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/${TAG}_gpu_tests.log | tail -8
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 1000 python -u bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; tail -25 gpurun_out/${TAG}_bench.err; head -c 1500 gpurun_out/${TAG}_bench.json; exit $rc
