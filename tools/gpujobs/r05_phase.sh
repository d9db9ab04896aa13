#!/bin/bash
# round 5: per-phase host cycles of the timed C3 run (bt2x-align-phase: -DBT2X_PHASE_PROF)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05t}
timeout -k 10 900 python3 bench.py --steps 20 --warmup 5 --runs 1 --no-cpu --no-legs --no-rep-leg --no-replay \
  --aligner $GRAFT_REPO_ROOT/omp-bowtie2-prime_amd/bt2x/bt2x-align-phase > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"
cp /tmp/bt2x_bench_$(id -u)/rank0/align0.err gpurun_out/${TAG}_align0.err && grep PHASE gpurun_out/${TAG}_align0.err
exit $rc
