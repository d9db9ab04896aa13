"""GPU-free host logic of the C++ shims (include/bt2x_shims.hpp) against the reference's
own outputs: SeedHitsHip = searchAllSeedsFinalize + SeedResults::add + rankSeedHits
(aligner_seed.cpp:508-540, aligner_seed.h:603-641, 1000-1061), fed the reference's
recorded seed-kernel outputs (tests/golden/seeds_rep.txt.xz), compared with
tests/golden/rank_rep.txt.xz (oracle/refharness.cpp "rank")."""
import os
import subprocess

import pytest

import golden_io as g

EXE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "test_host")


@pytest.fixture(scope="module")
def host_exe():
    if not os.access(EXE, os.X_OK):
        subprocess.run(["make", "-C", os.path.dirname(EXE), "test_host"], check=True,
                       stdout=subprocess.DEVNULL)
    return EXE


def _unpack(name, tmp_path):
    dst = str(tmp_path / name.replace(".xz", ""))
    with g.open_text(os.path.join(g.GOLDEN, name)) as fi, open(dst, "w") as fo:
        fo.write(fi.read())
    return dst


def test_rank_seed_hits_matches_reference(host_exe, tmp_path):
    seeds = _unpack("seeds_rep.txt.xz", tmp_path)
    rank = _unpack("rank_rep.txt.xz", tmp_path)
    out = subprocess.run([host_exe, "rank", seeds, rank], check=True, capture_output=True, text=True).stdout
    got = out.splitlines()
    exp = [ln.rstrip("\n") for ln in open(rank) if ln[:1] in ("K", "A")]
    assert len(exp) > 10000
    assert len(got) == len(exp)
    bad = [(a, b) for a, b in zip(got, exp) if a != b]
    assert not bad, bad[:5]
    # the set covers repetitive hits, both strands, and multi-draw rankings
    ks = [ln.split() for ln in exp if ln[0] == "K"]
    assert sum(int(k[12]) > 0 for k in ks) > 500           # repTot
    assert sum(int(k[7]) > 0 and int(k[6]) > 0 for k in ks) > 20    # hits on both strands
