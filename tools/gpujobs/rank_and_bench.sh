# the seed-round vs reference rank golden GPU test, then the default bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_round.py \
  > gpurun_out/r03_rank_test.log 2>&1
rc=$?; echo "rank test rc=$rc"; tail -15 gpurun_out/r03_rank_test.log
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/gpujobs/bench_full.sh
