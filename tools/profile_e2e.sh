# rocprofv3 summaries of the default bench workload (the aligner's launch sequence replayed
# from HBM): kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in passes of their own.
# Run on the GPU box from the repo root; tools/pmc_traffic.py --replays 3 turns the output
# into profiles/<tag>_*.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/prof_kt.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/prof_fetch.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/prof_write.log 2>&1
