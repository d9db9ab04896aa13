#!/bin/bash
# SQ issue/wait counters of the bench replay with and without the DP walks (BT2X_DP_ABLATE=1).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d gpurun_out/prof_wsq0 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_wsq0.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d gpurun_out/prof_wsq1 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --replay-ablate 1 > gpurun_out/prof_wsq1.log 2>&1
