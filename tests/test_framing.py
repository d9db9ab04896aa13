"""Host framing (bt2x/framing.py) against the rectangles and windows the reference's
DynProgFramer / SwAligner::initRef produced for the DP golden sets."""
import os

import numpy as np
import pytest

import golden_io as g
import framing_ref as framing


def genome_codes():
    import lzma
    with lzma.open(os.path.join(g.GOLDEN, "rep.fa.xz"), "rb") as f:
        raw = f.read()
    out, cur = [], []
    for line in raw.split(b"\n"):
        if line.startswith(b">"):
            if cur:
                out.append(g.codes(b"".join(cur)))
            cur = []
        elif line:
            cur.append(line.strip())
    if cur:
        out.append(g.codes(b"".join(cur)))
    return out


@pytest.mark.parametrize("gold,maxhalf", [("dp_rep.txt.xz", 15), ("dp_rep_dpad12.txt.xz", 12)])
def test_framing_matches_reference(gold, maxhalf):
    case = g.DpCase(os.path.join(g.GOLDEN, gold))
    ref = genome_codes()
    P = case.probs
    rdlen = np.array([len(p["seq"]) for p in P])
    np.testing.assert_array_equal(framing.min_score(rdlen), [p["minsc"] for p in P])
    np.testing.assert_array_equal(framing.n_ceil(rdlen), [p["nceil"] for p in P])
    ms = framing.min_score(rdlen)
    r = framing.frame_rect([p["refoff"] for p in P], rdlen, [p["tlen"] for p in P],
                           framing.max_read_gaps(ms, rdlen), framing.max_ref_gaps(ms, rdlen), maxhalf)
    for k in ("refl", "refr", "triml", "corel", "corer"):
        np.testing.assert_array_equal(r[k], [p[k] for p in P], err_msg=k)
    reads = [g.codes(p["seq"]) for p in P]
    quals = [np.frombuffer(p["qual"], np.uint8) for p in P]
    rd, qu, rf, dp, keep = framing.build_dp_batch(ref, [p["tidx"] for p in P], [p["refoff"] for p in P],
                                                  [p["fw"] for p in P], reads, quals, maxhalf=maxhalf)
    assert keep.all()
    np.testing.assert_array_equal(dp, case.inp)
    np.testing.assert_array_equal(rf, case.refs)
    np.testing.assert_array_equal(rd, case.reads)
    np.testing.assert_array_equal(qu, case.quals)


def test_max_gaps_known_answers():
    # Scoring::maxRefGaps / maxReadGaps at the defaults (5+3 open, 3 extend)
    assert framing.max_read_gaps(-90, 150) == 28
    assert framing.max_read_gaps(-60, 100) == 18
    assert framing.max_read_gaps(-7, 10) == 0 and framing.max_read_gaps(-8, 10) == 1
    assert framing.max_read_gaps(-11, 10) == 2
