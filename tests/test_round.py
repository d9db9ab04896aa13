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


def _rank_rounds(tmp_path):
    """The rep fixture's (read, round) pairs as bt2x_round_in rows (the golden's seeds, RNG
    seeds and round offsets), with the golden's seed rows and rank records."""
    import numpy as np
    from bt2x import abi
    import seeds_ref as bseeds
    base = g.materialize_index("rep", str(tmp_path))
    case = g.SeedCase(os.path.join(g.GOLDEN, "rep_reads.fq.xz"), os.path.join(g.GOLDEN, "seeds_rep.txt.xz"))
    reads = g.read_fastq(os.path.join(g.GOLDEN, "rep_reads.fq.xz"))
    # S rows per (read, round), in file order (the order bt2x_seed_round expects per read)
    rows = {}
    with g.open_text(os.path.join(g.GOLDEN, "seeds_rep.txt.xz")) as f:
        k = 0
        for line in f:
            if line.startswith("S "):
                t = line.split()
                rows.setdefault((int(t[1]), int(t[2])), []).append(k)
                k += 1
    ranks = []
    with g.open_text(os.path.join(g.GOLDEN, "rank_rep.txt.xz")) as f:
        for line in f:
            t = line.split()
            if t and t[0] in ("K", "Z"):
                ranks.append(t)
    L = 22
    seed_sel, rin, exp = [], [], []
    offs = np.cumsum([0] + [2 * len(s) for _, s, _ in reads])
    for t in ranks:
        ridx, rnd = int(t[1]), int(t[2])
        rdlen = len(reads[ridx][1])
        ival = bseeds.interval(rdlen)
        nrounds = min(2, ival)
        offset = (ival * rnd) // nrounds
        sl = min(L, rdlen)
        num_offs = 1 + (rdlen - offset - sl) // ival if rdlen - offset > sl else 1
        sel = rows.get((ridx, rnd), [])
        r = np.zeros(1, dtype=abi.ROUND_IN)
        r["read_off"] = offs[ridx]
        r["seed0"] = len(seed_sel)
        r["nseeds"] = len(sel)
        r["num_offs"] = num_offs
        r["rdlen"] = rdlen
        r["interval"] = ival
        r["offset"] = offset
        r["seedlen"] = sl
        if t[0] == "K":
            assert int(t[4]) == num_offs
            r["rnd_last"] = int(t[3])
        else:
            r["rnd_last"] = (ridx * 2654435761 + rnd * 97 + 1) & 0xffffffff
        r["rnd_lastoff"] = 30                       # RandomSource::init (random_source.h:46-50)
        seed_sel += sel
        rin.append(r)
        exp.append(t)
    rin = np.concatenate(rin)
    sin = case.inp[np.array(seed_sel, dtype=np.int64)]
    return base, case, reads, rin, sin, exp


@pytest.mark.gpu
def test_round_kernel_vs_reference_rank_golden(tmp_path):
    """bt2x_seed_round against the reference's own rankSeedHits (tests/golden/rank_rep.txt.xz,
    oracle/refharness.cpp "rank": aligner_seed.h:1000-1061 with a RandomSource seeded per
    (read, round)).  Every read and round of the rep fixture runs through the kernel with
    the golden's seeds, the golden's RNG seed and maxelt 0 (prioritizeSATups then samples
    nothing, so the returned RNG state is the state after ranking): NO_HITS exactly where the
    reference found none, and SeedResults::nonzeroOffsets(), numElts() and the RandomSource
    state after rankSeedHits equal the reference's."""
    import numpy as np
    from bt2x import abi, lib
    base, case, reads, rin, sin, exp = _rank_rounds(tmp_path)
    n = len(rin)
    ctx = lib.Context(lib.Index(base, load_offs=True))
    out = ctx.seed_round(case.reads, sin, rin, np.zeros(0, dtype=abi.EXRANGE), 0)[0]
    # the same round with the seeds instantiated on the GPU (seeds == NULL): the golden's
    # seed rows are the reference's instantiateSeeds list, so every output is the same
    gen = ctx.seed_round(case.reads, None, rin, np.zeros(0, dtype=abi.EXRANGE), 0)[0]
    ctx.close()
    keep = [f for f in out.dtype.names if f not in ("sat0", "elt0", "exr0")]   # arena offsets: atomics
    for f in keep:
        np.testing.assert_array_equal(gen[f], out[f], err_msg=f)
    bad, nk = [], 0
    for i, t in enumerate(exp):
        o = out[i]
        if t[0] == "Z":
            if o["status"] != 1:                    # BT2X_ROUND_NO_HITS
                bad.append((t[:3], "status", int(o["status"])))
            continue
        nk += 1
        got = (int(o["status"]), int(o["nonz"]), int(o["num_elts"]), int(o["rnd_last"]))
        want = (0, int(t[5]), int(t[8]), int(t[13]))
        if got != want:
            bad.append((t[:3], got, want))
    assert nk > 5000 and not bad, (len(bad), bad[:5])


@pytest.mark.gpu
def test_round_refuses_a_wrong_gpu_seed_count(tmp_path):
    """bt2x_seed_round with seeds == NULL checks each in[r].nseeds against the seeds the GPU
    instantiates (a seed over an N is skipped, so the count depends on the read's bytes):
    a read containing an N with its count off by one either way makes the call return
    BT2X_E_ARG, and the context still answers the correct call exactly afterwards."""
    import numpy as np
    from bt2x import abi, lib
    base, case, reads, rin, sin, exp = _rank_rounds(tmp_path)
    ctx = lib.Context(lib.Index(base, load_offs=True))
    noexr = np.zeros(0, dtype=abi.EXRANGE)
    ref = ctx.seed_round(case.reads, None, rin, noexr, 0)[0]
    # a round of a read with an N inside a would-be seed window (fewer seeds than offsets)
    sel = None
    for i, r in enumerate(rin):
        o = int(r["read_off"])
        codes = case.reads[o: o + int(r["rdlen"])]
        if (codes > 3).any() and 0 < int(r["nseeds"]) < 2 * int(r["num_offs"]):
            sel = i
            break
    assert sel is not None, "the rep fixture has reads with N"
    for delta in (1, -1):
        bad = rin.copy()
        bad["nseeds"][sel] = int(bad["nseeds"][sel]) + delta
        # later reads' seeds move with the count, so the reads' seeds never overlap
        bad["seed0"][sel + 1:] = (bad["seed0"][sel + 1:].astype(np.int64) + delta).astype(np.uint64)
        with pytest.raises(lib.Bt2xError) as e:
            ctx.seed_round(case.reads, None, bad, noexr, 0)
        assert e.value.code == abi.E_ARG
    again = ctx.seed_round(case.reads, None, rin, noexr, 0)[0]
    ctx.close()
    for f in ("status", "nonz", "num_elts", "rnd_last", "nsat", "nelt", "nexr"):
        np.testing.assert_array_equal(again[f], ref[f], err_msg=f)
