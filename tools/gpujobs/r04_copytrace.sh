# The timed run's kernels and PCIe copies: bench.py makes the inputs (as the driver runs it),
# then rocprofv3 traces bt2x-align over the same files (kernel + memory-copy trace, stats)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-legs --no-replay-whole \
  > gpurun_out/r04ff_bench.json 2> gpurun_out/r04ff_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
W=/tmp/bt2x_bench_$(id -u)
BASE=$(ls $W/syn*.1.bt2l | head -1); BASE=${BASE%.1.bt2l}
FILES=$(python3 -c "
import glob,re
fs=glob.glob('$W/rank0/*_R150_*.fq')
w=sorted([f for f in fs if re.search(r'/w\d+_',f)],key=lambda f:int(re.search(r'/w(\d+)_',f).group(1)))
s=sorted([f for f in fs if re.search(r'/s\d+_',f)],key=lambda f:int(re.search(r'/s(\d+)_',f).group(1)))
print(','.join(w+s))")
echo "base $BASE"
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/r04ff -o run --output-format csv -- \
  $GRAFT_REPO_ROOT/omp-bowtie2-prime_amd/bt2x/bt2x-align -x $BASE -U $FILES -S /dev/null --dpad 12 --device 0 -p 16 \
  --slots 131072 --warmup-files 5 --metrics --stats > gpurun_out/r04ff_align.out 2> gpurun_out/r04ff_align.err
rc=$?; echo "rocprof rc=$rc"; grep -E "BT2X_TIMED|BT2X_GPU" gpurun_out/r04ff_align.err | tail -3
find gpurun_out/r04ff -name "*stats*" | head; exit $rc
