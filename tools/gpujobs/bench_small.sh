# bench.py on a reduced configuration (plumbing check), then the default C3 run
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --genome-mb 200 --reads 400000 --steps 2 --warmup 1 --replay-reads 100000 \
  --cpu-sample 40000 --cpu-sample-1t 4000 > gpurun_out/r03_bench_small.json 2> gpurun_out/r03_bench_small.err
echo "small rc=$?"; tail -3 gpurun_out/r03_bench_small.err; cat gpurun_out/r03_bench_small.json | head -c 3000
