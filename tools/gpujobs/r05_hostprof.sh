#!/bin/bash
# host profile of the real timed run on the box: bench.py's C3 timed run through
# bt2x-align-prof (the driver with tools/sprof.c linked in: SIGPROF sampling, written at exit)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05d}
SPROF_WAIT=1 SPROF_RAW=$GRAFT_REPO_ROOT/gpurun_out/${TAG}_sprof_raw.txt SPROF_OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG}_sprof_flat.txt \
timeout -k 10 900 python3 bench.py --steps ${STEPS:-40} --warmup 5 --runs 1 --no-cpu --no-legs --no-rep-leg --no-replay \
  --aligner $GRAFT_REPO_ROOT/omp-bowtie2-prime_amd/bt2x/bt2x-align-prof ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/${TAG}_bench.json; head -25 gpurun_out/${TAG}_sprof_flat.txt
echo "$GRAFT_REPO_ROOT" > gpurun_out/${TAG}_root.txt
exit $rc
