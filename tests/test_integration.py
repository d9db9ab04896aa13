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
