# seed-round sampling iteration: the round and e2e GPU tests, then a rocprofv3 kernel
# trace + stats of a short bench run (per-kernel durations of round_sample_kernel et al.)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r04x}
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_round.py tests/test_e2e.py tests/test_gpu_parity.py \
  > gpurun_out/${TAG}_round_tests.log 2>&1
rc=$?; echo "round/e2e tests rc=$rc"; tail -3 gpurun_out/${TAG}_round_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o run -- python3 bench.py --no-cpu --no-legs --steps 5 --warmup 2 ${BENCH_ARGS} > gpurun_out/${TAG}_kt.log 2>&1
rc=$?; echo "profile rc=$rc"; tail -3 gpurun_out/${TAG}_kt.log
f=$(find gpurun_out/${TAG}_kt -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -12 "$f" | cut -c1-200
exit $rc
