"""Multi-rank read sharding on CPU (gloo, world_size 2): the N>1 path of bench.py and
of a sharded run, minus the GPU.  Each rank searches its contiguous shard of the rep
golden reads' seeds with the CPU oracle; the union equals the single-process result
and the counter sum equals the single-process counters."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "omp-bowtie2-prime_amd"))
from bt2x import dist as bdist  # noqa: E402

WORKER = r'''
import os, sys
import numpy as np
sys.path[:0] = [os.path.join(sys.argv[1], "omp-bowtie2-prime_amd"), os.path.join(sys.argv[1], "tests")]
import torch.distributed as dist
from bt2x import dist as bdist
import golden_io as g, oracle_lib as ol
dist.init_process_group("gloo")
rank, world, _ = bdist.world()
base = g.materialize_index("rep", os.path.join(sys.argv[2], f"idx{rank}"))
case = g.SeedCase(os.path.join(g.GOLDEN, "rep_reads.fq.xz"), os.path.join(g.GOLDEN, "seeds_rep.txt.xz"))
lo, hi = bdist.shard_bounds(case.n, rank, world)
out, _ = ol.seed_search(ol.OracleIndex(base), case.reads, case.inp[lo:hi], True)
np.save(os.path.join(sys.argv[2], f"shard{rank}.npy"), out)
ctr = bdist.sum_counters({"seeds": hi - lo, "reported": int(out["need_reporting"].sum())}, dist)
t = bdist.max_over_ranks(float(rank + 1), dist)
if rank == 0:
    with open(os.path.join(sys.argv[2], "ctr.txt"), "w") as f:
        f.write(f"{ctr['seeds']} {ctr['reported']} {t}")
dist.destroy_process_group()
'''


def test_shard_bounds_partition():
    for n in (0, 1, 7, 64, 1000003):
        for w in (1, 2, 3, 8):
            spans = [bdist.shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        bdist.shard_bounds(10, 2, 2)
    assert bdist.rank_seed(3, 0) == 3 and bdist.rank_seed(3, 1) != bdist.rank_seed(3, 0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gloo_two_rank_sharded_seed_search(tmp_path):
    import golden_io as g
    import oracle_lib as ol
    case = g.SeedCase(os.path.join(g.GOLDEN, "rep_reads.fq.xz"), os.path.join(g.GOLDEN, "seeds_rep.txt.xz"))
    base = g.materialize_index("rep", str(tmp_path / "idx"))
    worker = tmp_path / "worker.py"
    worker.write_text(WORKER)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(worker), ROOT, str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    full, _ = ol.seed_search(ol.OracleIndex(base), case.reads, case.inp, True)
    got = np.concatenate([np.load(tmp_path / f"shard{k}.npy") for k in range(2)])
    assert got.tobytes() == full.tobytes()
    seeds, rep, t = open(tmp_path / "ctr.txt").read().split()
    assert int(seeds) == case.n and int(rep) == int(full["need_reporting"].sum())
    assert float(t) == 2.0
