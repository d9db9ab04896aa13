# round-3 final measurements: host-driver A/B on the C3 inputs, then rocprofv3 summaries of
# bench.py --no-cpu --no-replay-whole (kernel trace + stats; FETCH_SIZE; WRITE_SIZE; SQ
# counters, each pass its own run); tools/pmc_traffic.py --replays 4 turns them into profiles/
bash tools/gpujobs/host_ab.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o run -- python3 bench.py --no-cpu --no-replay-whole > gpurun_out/prof_kt.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_fetch -o run -- python3 bench.py --no-cpu --no-replay-whole > gpurun_out/prof_fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_write -o run -- python3 bench.py --no-cpu --no-replay-whole > gpurun_out/prof_write.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/prof_sq -o run -- python3 bench.py --no-cpu --no-replay-whole > gpurun_out/prof_sq.log 2>&1
rc=$?; echo "profile rc=$rc"; tail -2 gpurun_out/prof_kt.log; ls gpurun_out/prof_kt gpurun_out/prof_sq 2>/dev/null | head; exit $rc
