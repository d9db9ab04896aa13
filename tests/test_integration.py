"""The reference-side drop-in compiled against the reference itself.

include/bt2x_ref_glue.hpp holds the two patches INTEGRATION.md applies -- the body of
MultiSeedAligner::searchAllSeedsDoAll (aligner_seed.cpp:674-725) and the SwAligner ->
SwResult translation in SwDriver::extendSeeds (aligner_sw_driver.cpp:481-538) -- over
include/bt2x_shims.hpp.  tests/cpp/ref_glue_compile.cpp instantiates them with the real
BTDnaString, BTString, Scoring, BitPairReference, DPRect, RandomSource, SwResult/AlnRes
and SeedAlignerSearchParams/Data, inside the reference's own translation unit
(bowtie2-align.cpp) and compile definitions (oracle/Makefile).  Needs /root/reference
(this container; the GPU box has none): skipped elsewhere.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


@pytest.mark.skipif(not os.path.isfile(os.path.join(REF, "aligner_sw.h")), reason="reference sources absent")
def test_glue_compiles_against_reference_types():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "glue_check"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]


def test_integration_md_uses_the_compiled_glue():
    """The patches INTEGRATION.md shows are the compiled ones (no hand-copied variants)."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert "bt2x::glue::search_all_seeds(" in text and "bt2x::glue::to_swresult(" in text
    glue = open(os.path.join(ROOT, "include", "bt2x_ref_glue.hpp")).read()
    for fn in ("search_all_seeds", "to_swresult"):
        assert re.search(r"\b" + fn + r"\(", glue)
    # every SwAligner call INTEGRATION.md shows is one the compile check makes
    check = open(os.path.join(ROOT, "tests", "cpp", "ref_glue_compile.cpp")).read()
    for call in ("swa.initRead(rd.patFw, rd.patRc, rd.qual, rd.qualRev, rdlen, sc)", "swa.align(best)",
                 "swa.nextAlignment(v, (int64_t)minsc, rnd)", "swa.done()"):
        assert call in check


# ------------------------------------------------------------------ the drop-in, executed
# oracle/ref_glue_build.py builds the reference aligner itself with the two patches
# applied -- its searchAllSeedsDoAll and its SwAligner (initRead / initRef / align /
# nextAlignment / done) routed through libbt2x.so via include/bt2x_ref_glue.hpp and
# include/bt2x_shims.hpp -- into oracle/_ref/bowtie2-align-l-bt2x[-i16] (built here, where
# /root/reference exists; the binaries travel to the GPU box).  Its SAM, alignment summary
# and warnings must equal the stock reference's (the committed e2e goldens).
PATCHED = {"u8": os.path.join(ROOT, "oracle", "_ref", "bowtie2-align-l-bt2x"),
           "i16": os.path.join(ROOT, "oracle", "_ref", "bowtie2-align-l-bt2x-i16")}
DROPIN_SETS = [("e2e_rep", "rep", "rep_reads.fq", [], "u8"),
               ("e2e_tandem", "tandem", "tandem_reads.fq", [], "u8"),
               ("e2e_rep_dpad12", "rep", "rep_reads.fq", ["--dpad", "12"], "u8"),
               ("e2e_rep_i16", "rep", "rep_reads.fq", ["--no-sse8"], "i16")]


def _run_patched(tmp_path, binary, name, idx, fq, opts):
    import lzma
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import golden_io as g
    from test_e2e import check_summary, sam_records
    if not os.access(binary, os.X_OK):
        pytest.skip("oracle/_ref/ has no patched reference build (needs /root/reference where it is built)")
    base = g.materialize_index(idx, str(tmp_path))
    reads = tmp_path / fq
    with lzma.open(os.path.join(g.GOLDEN, fq + ".xz"), "rb") as f:
        reads.write_bytes(f.read())
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run([binary, "-x", base, "-U", str(reads)] + opts, capture_output=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    with lzma.open(os.path.join(g.GOLDEN, name + ".sam.xz"), "rb") as f:
        exp = sam_records(f.read())
    got = sam_records(r.stdout)
    bad = [(a, b) for a, b in zip(got, exp) if a != b]
    assert len(got) == len(exp) and not bad, (len(got), len(exp), bad[:1])
    check_summary(b"\n".join(ln for ln in r.stderr.split(b"\n") if not ln.startswith(b"Timer:")), name)


@pytest.mark.gpu
@pytest.mark.parametrize("name,idx,fq,opts,build", DROPIN_SETS, ids=[s[0] for s in DROPIN_SETS])
def test_patched_reference_aligner_on_gpu(tmp_path, name, idx, fq, opts, build):
    _run_patched(tmp_path, PATCHED[build], name, idx, fq, opts)


@pytest.mark.parametrize("name,idx,fq,opts,build", DROPIN_SETS, ids=[s[0] for s in DROPIN_SETS])
def test_patched_reference_glue_on_cpu(tmp_path, name, idx, fq, opts, build):
    """The same patched aligner with the C-ABI answered by the CPU oracle
    (oracle/bt2x_abi_oracle.cpp, oracle/ref_glue_build.py --cpu): the glue's hand-over of
    the reference's seed batch and SwAligner state is checked in the CPU suite, so a glue
    fault is told apart from a kernel fault."""
    _run_patched(tmp_path, PATCHED[build] + "-cpu", name, idx, fq, opts)
