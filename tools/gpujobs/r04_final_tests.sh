set -o pipefail
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04z_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -eq 0 ]; then
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04z_smoke.log 2>&1; echo "smoke rc=$?"
fi
tail -5 gpurun_out/r04z_gpu_tests.log
