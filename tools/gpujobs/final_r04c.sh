# round-4 final C: WRITE_SIZE and the SQ counters, each in a pass of its own
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
B="bench.py --no-cpu --no-legs --no-replay-whole"
timeout -k 10 550 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_write -o run -- python3 $B > gpurun_out/prof_write.log 2>&1 && \
timeout -k 10 550 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/prof_sq -o run -- python3 $B > gpurun_out/prof_sq.log 2>&1
rc=$?; echo "profile C rc=$rc"; tail -2 gpurun_out/prof_sq.log; exit $rc
