#!/bin/bash
# round 6: the N = 2 bench path rehearsed on the box's one GPU (both ranks on device 0):
# per-rank CPU sets inside the GPU's node, summed counters, max-over-ranks time
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${T:-r06n2}
BT2X_BENCH_DEVICE=0 timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
	--master-port 29555 bench.py --gpus 2 --steps 20 --warmup 5 --runs 1 --no-cpu --no-legs --no-rep-leg --no-replay \
	> gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/${T}_bench.err; exit $rc; }
python3 -c "
import json
for ln in open('gpurun_out/${T}_bench.json'):
    if ln.startswith('{'): d = json.loads(ln)
c = d['config']
print(d['value'], d['n_gpus'], d['end_to_end']['summary'][0], c['host_threads'], c['host_threads_note'], c['host_cpus'], c['host_cpus_note'])"
