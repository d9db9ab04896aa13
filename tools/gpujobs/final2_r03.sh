# round-3 final tree: rocprofv3 summaries of bench.py --no-cpu --no-replay-whole (kernel trace +
# stats; FETCH_SIZE; WRITE_SIZE; SQ counters), then the default bench and smoke()
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o run -- python3 bench.py --no-cpu --no-replay-whole > gpurun_out/prof_kt.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_fetch -o run -- python3 bench.py --no-cpu --no-replay-whole > gpurun_out/prof_fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_write -o run -- python3 bench.py --no-cpu --no-replay-whole > gpurun_out/prof_write.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/prof_sq -o run -- python3 bench.py --no-cpu --no-replay-whole > gpurun_out/prof_sq.log 2>&1
rc=$?; echo "profile rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke_final.log 2>&1; echo "smoke rc=$?"
bash tools/gpujobs/bench_full.sh
