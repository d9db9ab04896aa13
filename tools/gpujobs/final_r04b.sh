# round-4 final B: rocprofv3 summaries of bench.py --no-cpu --no-legs --no-replay-whole:
# kernel trace + stats, then FETCH_SIZE in a pass of its own (tools/pmc_traffic.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
B="bench.py --no-cpu --no-legs --no-replay-whole"
timeout -k 10 550 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o run -- python3 $B > gpurun_out/prof_kt.log 2>&1 && \
timeout -k 10 550 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_fetch -o run -- python3 $B > gpurun_out/prof_fetch.log 2>&1
rc=$?; echo "profile B rc=$rc"; tail -2 gpurun_out/prof_kt.log; exit $rc
