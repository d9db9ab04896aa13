# GPU tests, then the bench's multi-rank path rehearsed with 2 ranks on this box's one GPU
# (reduced workload; BT2X_BENCH_DEVICE pins both ranks to device 0)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r03_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r03_gpu_tests.log | tail -4
case $rc in 0|1) ;; *) exit $rc;; esac
BT2X_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --genome-mb 200 --reads 400000 --steps 2 --warmup 1 --replay-reads 100000 \
  > gpurun_out/r03_bench_n2.json 2> gpurun_out/r03_bench_n2.err
rc=$?; echo "bench n2 rc=$rc"; tail -5 gpurun_out/r03_bench_n2.err; head -c 800 gpurun_out/r03_bench_n2.json
