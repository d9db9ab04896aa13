#!/bin/bash
# SQ counters + FETCH/WRITE for the current kernels on a short bench run.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD \
  --kernel-trace --output-format csv -d gpurun_out/prof_sq -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/prof_sq.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_fetch -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/prof_fetch.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_write -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/prof_write.log 2>&1
