#!/bin/bash
# Instruction-cache and issue counters of the DP fill (BT2X_DP_ABLATE=1: fill + candidate order, no walk) on the bench replay.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
(timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true) && \
BT2X_DP_ABLATE=1 timeout -s KILL 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVES SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/prof_ic -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_ic.log 2>&1 && \
BT2X_DP_ABLATE=1 timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/prof_sq -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_sq.log 2>&1
