#!/bin/bash
# Development tool (GPU box): after a bench.py run has left its genome index and reads
# under /tmp/bt2x_bench_$UID, time bt2x-align end to end under several option sets.
#   tools/e2e_sweep.sh "<opts 1>" "<opts 2>" ...
set -o pipefail
W=/tmp/bt2x_bench_$(id -u)
ALIGN=$(dirname "$0")/../omp-bowtie2-prime_amd/bt2x/bt2x-align
for opts in "$@"; do
  echo "== $opts"
  # an option set may start with VAR=value environment settings
  envs=()
  while [[ "$opts" =~ ^([A-Z_]+=[^ ]*)\ (.*)$ ]]; do envs+=("${BASH_REMATCH[1]}"); opts="${BASH_REMATCH[2]}"; done
  timeout -k 10 300 env "${envs[@]}" "$ALIGN" -x "$W/syn1000000000_s2024" -U "$W/rank0/reads.fq" -S "$W/sweep.sam" --dpad 12 \
      -p "${OMP_NUM_THREADS:-16}" --stats $opts 2>&1 | grep -E "BT2X_STATS|BT2X_RUSAGE|BT2X_GPU|overall" || exit 1
done
