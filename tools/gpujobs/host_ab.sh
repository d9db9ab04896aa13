# host-driver A/B on the bench's C3 inputs: bt2x-align (this tree) vs bt2x-align-prev, alternated
# (bt2x-align-prev: the previous host driver, built by hand from an older commit with the same g++ line as host/Makefile)
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --no-cpu --no-replay > gpurun_out/hab_bench.json 2> gpurun_out/hab_bench.err
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/hab_bench.err; [ $rc -eq 0 ] || exit $rc
W=/tmp/bt2x_bench_$(id -u)
FQ=$(ls $W/rank0/w0_*.fq),$(ls $W/rank0/s*_*.fq | sort -t s -k2 -n | paste -sd,)
for i in 1 2; do for b in bt2x-align bt2x-align-prev; do
  timeout -k 10 200 omp-bowtie2-prime_amd/bt2x/$b -x $W/syn3100000000_s2024 -U $FQ -S /tmp/hab.sam --dpad 12 -p 16 \
    --slots 131072 --warmup-files 1 --metrics --stats > /dev/null 2> gpurun_out/hab_$b.$i.err
  echo "$b $i rc=$? $(grep -o 't_align=[0-9.]*' gpurun_out/hab_$b.$i.err | head -1) $(grep BT2X_RUSAGE_ALIGN gpurun_out/hab_$b.$i.err)"
done; done
