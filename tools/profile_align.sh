#!/bin/bash
# Kernel + memory-copy trace of the end-to-end aligner on the bench workload: bench.py
# writes the data, then bt2x-align runs under rocprofv3 (the profiler does not follow
# bench.py's child processes).  Output: gpurun_out/prof_align/.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python3 bench.py --prep-only > gpurun_out/prep.log 2>&1 && \
read -r _ BASE FQ < <(grep '^BT2X_DATA' gpurun_out/prep.log) && \
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_align -o run -- \
  omp-bowtie2-prime_amd/bt2x/bt2x-align -x "$BASE" -U "$FQ" -S /tmp/bt2x_prof.sam --dpad 12 -p 16 --slots 131072 --lookahead 8 --stats \
  > gpurun_out/prof_align.log 2>&1
