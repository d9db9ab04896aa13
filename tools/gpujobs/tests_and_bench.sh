# the GPU test suite, then the default bench (stops after a GPU fault/timeout)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r03_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r03_gpu_tests.log | tail -8
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/gpujobs/bench_full.sh
