set -o pipefail
( nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; free -g | head -2; df -h /tmp /dev/shm | cat; lscpu | grep -E "Model name|Flags" | cut -c1-200; echo OMP=$OMP_NUM_THREADS ) > gpurun_out/r03c_boxinfo.txt 2>&1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03c_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03c_smoke.log 2>&1; echo "smoke rc=$?"
fi
tail -5 gpurun_out/r03c_gpu_tests.log
