#!/bin/bash
# round-5 final: the driver's bench command (N=1) on the final tree
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 1150 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05_bench.json 2> gpurun_out/r05_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/r05_bench.json; ps -eo pid,ppid,comm | grep -c bt2x-align || true
exit $rc
