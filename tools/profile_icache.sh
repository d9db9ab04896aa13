cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; \
timeout -k 10 400 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d gpurun_out/prof_ic -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/prof_ic.log 2>&1
