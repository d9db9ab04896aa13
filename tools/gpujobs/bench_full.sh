# the default bench.py run (config C3: 3.1 Gbp synthetic genome, 10M x 150 bp, --dpad 12)
mkdir -p gpurun_out
timeout -k 10 1000 python -u bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err
rc=$?; echo "bench rc=$rc"; tail -25 gpurun_out/r03_bench.err; head -c 1500 gpurun_out/r03_bench.json; exit $rc
