# bench setup (C3 genome, index, reads) + the timed run, then bt2x-align over the same
# step files at other --slots / -p / --lookahead settings (end-to-end t_align each)
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --no-cpu --no-replay > gpurun_out/r03_sweep_bench.json 2> gpurun_out/r03_sweep_bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r03_sweep_bench.err; [ $rc -eq 0 ] || exit $rc
W=/tmp/bt2x_bench_$(id -u); B=$W/syn3100000000_s2024
U=$(ls $W/rank0/w0_*.fq),$(ls $W/rank0/s*_*.fq | sort -V | paste -sd,)
for cfg in "--slots 65536" "--slots 131072" "--slots 524288" "--slots 262144 --lookahead 4" "--slots 262144 --lookahead 16" "--slots 262144 -p 15"; do
  timeout -k 10 120 omp-bowtie2-prime_amd/bt2x/bt2x-align -x $B -U $U -S $W/sweep.sam --dpad 12 -p 16 --warmup-files 1 --metrics --stats $cfg \
    2> gpurun_out/sweep.err > /dev/null
  rc=$?; echo "$cfg rc=$rc $(grep -o 't_align=[0-9.]*' gpurun_out/sweep.err | head -1) $(grep -o 'user=[0-9.]*' gpurun_out/sweep.err | tail -1) $(grep BT2X_GPU gpurun_out/sweep.err | cut -c1-160)"
  [ $rc -eq 0 ] || exit $rc
done
rm -f $W/sweep.sam
