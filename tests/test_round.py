"""The seed round (searchAllSeedsFinalize + rankSeedHits + prioritizeSATups + the rows
extendSeeds resolves) that bt2x_seed_round runs on the GPU, against the host driver's
restatement host_round, which tests/test_e2e.py pins to the reference's SAM.

tests/cpp/test_round checks every read of a fixture for two seed rounds (the second
with the first's exRange) and maxelt 400/1/3/7/20/60 (small values force RowSampler and
Random1toN sampling).  Fixtures: the committed rep and tandem sets, and a generated
high-repeat genome whose seed ranges exceed 128 elements, so Random1toN runs in its
seen-list mode and converts to a swap list (random_util.h:32-230).

* `-m "not gpu"`: csrc/round_core.h compiled for the host (the code the kernel runs).
* `-m gpu`: the kernel through the C-ABI, one launch per maxelt.
"""
from __future__ import annotations

import lzma
import os
import subprocess
import sys

import pytest

import golden_io as g

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "omp-bowtie2-prime_amd"))
TEST = os.path.join(ROOT, "tests", "cpp", "test_round")


@pytest.fixture(scope="module")
def sets(tmp_path_factory):
    import simdata as sd
    from bt2x import lib
    d = tmp_path_factory.mktemp("round")
    out = []
    for idx, fq in (("rep", "rep_reads.fq"), ("tandem", "tandem_reads.fq")):
        base = g.materialize_index(idx, str(d))
        p = d / fq
        with lzma.open(os.path.join(g.GOLDEN, fq + ".xz"), "rb") as fi:
            p.write_bytes(fi.read())
        out.append((idx, base, str(p)))
    # high-repeat genome: 8 families at ~250 copies each, 2 % divergence
    chroms = sd.gen_genome(1_000_000, nchrom=2, seed=5, repeat_frac=0.6, n_runs_per_mb=0)
    fa = d / "hirep.fa"
    sd.write_fasta(str(fa), chroms)
    base = str(d / "hirep")
    lib.build_index(str(fa), base)
    reads = sd.sim_reads(chroms, 1500, 100, seed=9) + sd.sim_reads(chroms, 500, 150, seed=10)
    fq = d / "hirep.fq"
    sd.write_fastq(str(fq), reads)
    out.append(("hirep", base, str(fq)))
    return out


def run(args):
    assert os.access(TEST, os.X_OK), "build first: make -C tests/cpp"
    r = subprocess.run([TEST] + args, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:] + r.stdout[-500:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("round ")][-1]
    return {k: int(v) for k, v in (t.split("=") for t in line.split()[1:])}


def test_round_core_matches_host(sets):
    for name, base, fq in sets:
        st = run([base, fq, "--core"])
        assert st["mismatches"] == 0 and st["cases"] > 1000, (name, st)
        if name == "hirep":
            assert st["sampled"] > 1000 and st["seenmode"] > 0 and st["converted"] > 0, st


@pytest.mark.gpu
def test_round_kernel_matches_host(sets):
    for name, base, fq in sets:
        st = run([base, fq, "--gpu"])
        assert st["mismatches"] == 0 and st["cases"] > 1000, (name, st)
