#!/bin/bash
# round 5: the full -m gpu suite + smoke, then a short bench run; processes of this user
# still alive after bench.py are listed (run.procs_at_end)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05a}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${TAG}_smoke.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$BENCH" ]; then
  timeout -k 10 900 python3 bench.py $BENCH > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/${TAG}_bench.json
  sleep 2; ps -u $(id -u) -o pid,ppid,pgid,etime,cmd > gpurun_out/${TAG}_ps_after.txt; cat gpurun_out/${TAG}_ps_after.txt | head -20
fi
exit $rc
