#!/bin/bash
# Kernel traces of the bench replay with and without the DP walk (BT2X_DP_ABLATE=1), same box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ab0 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_ab0.log 2>&1 && \
BT2X_DP_ABLATE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ab1 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_ab1.log 2>&1
