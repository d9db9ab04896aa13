#!/bin/bash
# SQ instruction-mix pass on the default bench workload (SALU/VALU/LDS/branch counts and waits).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY \
  --kernel-trace --output-format csv -d gpurun_out/prof_sq2 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_sq2.log 2>&1
