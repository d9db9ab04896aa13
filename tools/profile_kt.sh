#!/bin/bash
# Kernel-trace + stats of a short bench run (per-kernel average durations).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/prof_kt2.log 2>&1
