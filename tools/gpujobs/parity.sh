set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03b_parity.log 2>&1
echo "pytest rc=$?"
grep -E "PASSED|FAILED|ERROR" gpurun_out/r03b_parity.log | sed 's/.*:://' | cut -c1-150
