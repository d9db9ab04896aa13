# GPU tests, then bench setup + a sweep of bt2x-align settings on the C3 step files
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r03_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r03_gpu_tests.log | tail -6
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python -u bench.py --no-cpu --no-replay --slots 131072 > gpurun_out/r03_sweep_bench.json 2> gpurun_out/r03_sweep_bench.err
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/r03_sweep_bench.err; [ $rc -eq 0 ] || exit $rc
W=/tmp/bt2x_bench_$(id -u); B=$W/syn3100000000_s2024
U=$(ls $W/rank0/w0_*.fq),$(ls $W/rank0/s*_*.fq | sort -V | paste -sd,)
for cfg in "--slots 131072" "--slots 131072 --lookahead 12" "--slots 131072 --lookahead 16" "--slots 98304" "--slots 98304 --lookahead 16" "--slots 131072"; do
  timeout -k 10 120 omp-bowtie2-prime_amd/bt2x/bt2x-align -x $B -U $U -S $W/sweep.sam --dpad 12 -p 16 --warmup-files 1 --metrics --stats $cfg \
    2> gpurun_out/sweep.err > /dev/null
  rc=$?; echo "$cfg rc=$rc $(grep -o 't_align=[0-9.]*' gpurun_out/sweep.err | head -1) $(grep -o 'user=[0-9.]*' gpurun_out/sweep.err | tail -1) $(grep BT2X_GPU gpurun_out/sweep.err | cut -c1-200)"
  [ $rc -eq 0 ] || exit $rc
done
rm -f $W/sweep.sam
