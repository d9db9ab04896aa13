"""End-to-end parity: FASTQ in, SAM out, against the reference aligner's own SAM.

Goldens (tests/golden/e2e_*.sam.xz) are the output of the reference's bowtie2-align-l
(1 thread) on the committed lambda and rep fixtures, as sorted, @PG-less records
(tools/make_golden.py e2e; the reference's own comparison methodology, scripts/sim
Sim.pm).  Sets: the lambda example reads (2000 records, 40-2561 bp, most unaligned by
the fork's length limits), and 3660 rep reads of 12-160 bp (repeats, N runs, indels)
under the default scoring, --dpad 12 and a non-default scoring scheme.

* `-m "not gpu"`: tests/cpp/test_e2e_oracle — the product's host driver
  (omp-bowtie2-prime_amd/host: per-read coroutine, prioritizeSATups, extendSeeds,
  reporting, MAPQ, SAM, the F11 edit-buffer replay) with the CPU oracle standing in for
  the three kernels.  This pins the host logic without a GPU.
* `-m gpu`: the product binary bt2x-align (host driver over libbt2x.so, every seed
  search / SA resolution / DP on the MI355X).
"""
from __future__ import annotations

import lzma
import os
import subprocess

import pytest

import golden_io as g

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALIGN = os.path.join(ROOT, "omp-bowtie2-prime_amd", "bt2x", "bt2x-align")
ORACLE_DRIVER = os.path.join(ROOT, "tests", "cpp", "test_e2e_oracle")
ALT_OPTS = ["--mp", "5,1", "--np", "2", "--rdg", "4,2", "--rfg", "6,3", "--gbar", "2"]
SETS = [("e2e_lambda", "lambda_virus", "lambda_longreads.fq", []),
        ("e2e_rep", "rep", "rep_reads.fq", []),
        ("e2e_rep_dpad12", "rep", "rep_reads.fq", ["--dpad", "12"]),
        ("e2e_rep_alt", "rep", "rep_reads.fq", ALT_OPTS),
        ("e2e_tandem", "tandem", "tandem_reads.fq", []),
        ("e2e_tandem_dpad12", "tandem", "tandem_reads.fq", ["--dpad", "12"])]


def sam_records(data: bytes) -> list[bytes]:
    lines = [ln for ln in data.split(b"\n") if ln and not ln.startswith(b"@PG")]
    return [ln for ln in lines if ln.startswith(b"@")] + sorted(ln for ln in lines if not ln.startswith(b"@"))


@pytest.fixture(scope="module")
def fixtures(tmp_path_factory):
    d = tmp_path_factory.mktemp("e2e")
    out = {}
    for _, idx, fq, _ in SETS:
        if idx not in out:
            out[idx] = g.materialize_index(idx, str(d))
        if fq not in out:
            p = d / fq
            with lzma.open(os.path.join(g.GOLDEN, fq + ".xz"), "rb") as fi:
                p.write_bytes(fi.read())
            out[fq] = str(p)
    return out


def check(cmd: list[str], golden: str):
    r = subprocess.run(cmd, capture_output=True, timeout=600)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    got = sam_records(r.stdout)
    with lzma.open(os.path.join(g.GOLDEN, golden + ".sam.xz"), "rb") as f:
        exp = sam_records(f.read())
    bad = [(a, b) for a, b in zip(got, exp) if a != b]
    assert len(got) == len(exp) and not bad, \
        f"{len(bad)} of {len(exp)} records differ; first:\n ours {bad[0][0][:300]!r}\n ref  {bad[0][1][:300]!r}" \
        if bad else f"{len(got)} records vs {len(exp)}"
    return got, r.stderr


@pytest.mark.parametrize("name,idx,fq,opts", SETS, ids=[s[0] for s in SETS])
def test_host_driver_vs_reference_sam(fixtures, name, idx, fq, opts):
    """Host driver + CPU oracle kernels == the reference's SAM (no GPU)."""
    assert os.access(ORACLE_DRIVER, os.X_OK), "build first: make -C tests/cpp"
    got, err = check([ORACLE_DRIVER, fixtures[idx], fixtures[fq], "--slots", "777", "-p", "4"] + opts, name)
    n_al = sum(1 for ln in got if not ln.startswith(b"@") and ln.split(b"\t")[1] != b"4")
    # (150 bp reads need --dpad <= 12 to fit ALN_MAX_COLS: SURVEY F2)
    assert n_al > {"lambda_virus": 400, "rep": 2000, "tandem": 1400}[idx]
    if idx == "tandem":
        # the fixture's point: -M tightens minsc between nextAlignment calls of one DP
        # problem (records consumed after a tightening in the same problem)
        tight = int(err.split(b"tight_recs=")[1].split()[0])
        assert tight > 100, tight


@pytest.mark.parametrize("name,idx,fq,opts", [SETS[1], SETS[4]], ids=[SETS[1][0], SETS[4][0]])
def test_host_driver_vs_reference_sam_three_requests(fixtures, name, idx, fq, opts):
    """The same with every seed round as seed search + host ranking/prioritization + SA
    resolution (the path a read takes when the GPU round hands it back)."""
    check([ORACLE_DRIVER, fixtures[idx], fixtures[fq], "--slots", "777", "-p", "4", "--no-gpu-round"] + opts, name)


def test_host_driver_slot_count_invariance(fixtures):
    """Results do not depend on how many reads are in flight."""
    outs = []
    for slots in ("1", "64", "5000"):
        r = subprocess.run([ORACLE_DRIVER, fixtures["rep"], fixtures["rep_reads.fq"], "--slots", slots, "-p", "3"],
                           capture_output=True, timeout=600, check=True)
        outs.append(sam_records(r.stdout))
    assert outs[0] == outs[1] == outs[2]


@pytest.mark.gpu
@pytest.mark.parametrize("name,idx,fq,opts", SETS, ids=[s[0] for s in SETS])
def test_bt2x_align_vs_reference_sam(fixtures, name, idx, fq, opts):
    """The product binary (kernels on the MI355X) == the reference's SAM."""
    check([ALIGN, "-x", fixtures[idx], "-U", fixtures[fq], "--slots", "1000"] + opts, name)


def test_host_driver_lookahead_invariance(fixtures):
    """DP lookahead (problems posed ahead of need and memoised by DpKey) changes the
    number of launches, never the records."""
    outs = []
    for la in ("1", "8", "64"):
        r = subprocess.run([ORACLE_DRIVER, fixtures["rep"], fixtures["rep_reads.fq"], "--slots", "3000", "-p", "3",
                            "--dpad", "12", "--lookahead", la], capture_output=True, timeout=600, check=True)
        outs.append(sam_records(r.stdout))
    assert outs[0] == outs[1] == outs[2]
    with lzma.open(os.path.join(g.GOLDEN, "e2e_rep_dpad12.sam.xz"), "rb") as f:
        assert outs[0] == sam_records(f.read())
