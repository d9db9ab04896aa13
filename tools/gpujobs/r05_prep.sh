#!/bin/bash
# round_prep_kernel after the strand-bitmask ranking: the round's GPU tests and the e2e
# tests, then the kernel trace of the C3 bench (no legs) as in final_r05a.sh
T=${T:-r05x}; cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_round.py tests/test_e2e.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
B="bench.py --no-cpu --no-legs --no-rep-leg --no-replay-whole --runs 1"
timeout -k 10 550 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o run -- python3 $B > gpurun_out/${T}_kt.log 2>&1
rc=$?; tail -c 300 gpurun_out/${T}_kt.log; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/${T}_kt -name '*kernel_stats.csv' | head -1); cp $f gpurun_out/${T}_kernel_stats.csv
grep -i "round_\|seed_kernel\|sa_resolve" gpurun_out/${T}_kernel_stats.csv | cut -c1-160
rm -rf gpurun_out/${T}_kt
