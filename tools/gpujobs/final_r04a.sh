# round-4 final A: the bench line as the driver runs it (CPU baseline, parity, C2/C5 legs),
# then a rocprofv3 kernel trace + stats of the C2 leg's aligner run (the i16 DP kernel)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 1000 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r04_bench.err; head -c 400 gpurun_out/r04_bench.json; echo
[ $rc -eq 0 ] || exit $rc
WD=/tmp/bt2x_bench_$(id -u)
C2=$(ls $WD/rank0/c2_1_*_R100.fq | head -1)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_c2 -o run -- ./omp-bowtie2-prime_amd/bt2x/bt2x-align -x $WD/ecoli -U $C2 -S /dev/null --no-sse8 -p 16 --stats > gpurun_out/r04_c2.log 2>&1
rc=$?; echo "c2 profile rc=$rc"; tail -2 gpurun_out/r04_c2.log; head -8 gpurun_out/r04_c2/run_kernel_stats.csv | cut -c1-160
exit $rc
