# bench setup + timed run, then bt2x-align with the DP wave-kernel threshold swept
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --no-cpu --no-replay > gpurun_out/r03_sweep_bench.json 2> gpurun_out/r03_sweep_bench.err
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/r03_sweep_bench.err; [ $rc -eq 0 ] || exit $rc
W=/tmp/bt2x_bench_$(id -u); B=$W/syn3100000000_s2024
U=$(ls $W/rank0/w0_*.fq),$(ls $W/rank0/s*_*.fq | sort -V | paste -sd,)
for sp in 0 4 8 6 0 4; do
  BT2X_DP_SPREAD=$sp timeout -k 10 120 omp-bowtie2-prime_amd/bt2x/bt2x-align -x $B -U $U -S $W/sweep.sam --dpad 12 -p 16 --warmup-files 1 --metrics --stats \
    2> gpurun_out/sweep.err > /dev/null
  rc=$?; echo "spread=$sp rc=$rc $(grep -o 't_align=[0-9.]*' gpurun_out/sweep.err | head -1) $(grep -o 'user=[0-9.]*' gpurun_out/sweep.err | tail -1) $(grep BT2X_GPU gpurun_out/sweep.err | cut -c1-200)"
  [ $rc -eq 0 ] || exit $rc
done
rm -f $W/sweep.sam
