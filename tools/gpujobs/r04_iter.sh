# one DP iteration: GPU tests, DP replay at cohort and whole-file shapes, then the bench as
# the driver runs it
mkdir -p gpurun_out
TAG=${TAG:-r04x}
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for s in 65536 1048576; do
timeout -k 10 400 python -u tools/dp_replay.py --slots $s "" ${DP_CFGS} > gpurun_out/${TAG}_dpreplay_$s.log 2>&1
rc=$?; echo "slots $s rc=$rc"; grep -E "config|launches|Error|error" gpurun_out/${TAG}_dpreplay_$s.log | tail -9
[ $rc -eq 0 ] || exit $rc
done
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 1000 python -u bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; tail -4 gpurun_out/${TAG}_bench.err; head -c 600 gpurun_out/${TAG}_bench.json; exit $rc
