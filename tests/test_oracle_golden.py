"""Pin the CPU restatement (oracle/bt2x_oracle.c) against golden vectors dumped by the
reference's own code (oracle/refharness.cpp via tools/make_golden.py).

The oracle must be bit-exact here before it is trusted as the checker of the HIP
kernels on the GPU box (where the reference does not exist)."""
import os

import numpy as np
import pytest

import golden_io as g
import oracle_lib as ol

SEED_SETS = [("lambda_virus", "lambda_longreads.fq.xz", "seeds_lambda.txt.xz"),
             ("rep", "rep_reads.fq.xz", "seeds_rep.txt.xz")]
DP_SETS = ["dp_rep.txt.xz", "dp_rep_dpad12.txt.xz", "dp_rep_alt.txt.xz"]
# the reference's i16 kernel (refharness-i16, a -DENABLE_I16 build): --no-sse8; --no-sse8
# with minimum scores below the u8 floor; and that build's default (u8 unless minsc < -254)
I16_DP_SETS = ["dp_rep_i16.txt.xz", "dp_rep_i16_wide.txt.xz", "dp_rep_i16_mix.txt.xz"]


def scoring_for(golden):
    sc = ol.default_scoring()
    for k, v in g.dp_header_scoring(golden).items():
        setattr(sc, k, v)
    ol.lib().bt2o_scoring_init.argtypes = [ol.ctypes.POINTER(g.abi.Scoring)]
    ol.lib().bt2o_scoring_init(ol.ctypes.byref(sc))
    return sc


@pytest.mark.parametrize("name,fq,gold", SEED_SETS)
def test_seed_search_matches_reference(golden_dir, name, fq, gold):
    base = g.materialize_index(name, str(golden_dir))
    idx = ol.OracleIndex(base)
    case = g.SeedCase(os.path.join(g.GOLDEN, fq), os.path.join(g.GOLDEN, gold))
    assert case.n > 20000
    out, ctr = ol.seed_search(idx, case.reads, case.inp, do_extend=True)
    np.testing.assert_array_equal(out["need_reporting"], case.exp_rep)
    np.testing.assert_array_equal(out["topf"], case.exp_topf)
    np.testing.assert_array_equal(out["botf"], case.exp_botf)
    np.testing.assert_array_equal(out["nlex"], case.exp_nlex)
    assert ctr["n_lf1"] > 0


def test_rep_set_covers_multi_row_ranges(golden_dir):
    case = g.SeedCase(os.path.join(g.GOLDEN, "rep_reads.fq.xz"), os.path.join(g.GOLDEN, "seeds_rep.txt.xz"))
    rep = case.exp_rep == 1
    assert ((case.exp_botf - case.exp_topf)[rep] > 1).sum() > 1000      # mapBiLFEx path
    assert (case.exp_nlex[rep] > 0).sum() > 1000                        # extension path
    assert (case.exp_rep == 0).sum() > 1000                             # failing seeds


@pytest.mark.parametrize("gold", DP_SETS)
def test_dp_matches_reference(gold):
    path = os.path.join(g.GOLDEN, gold)
    case = g.DpCase(path)
    assert case.n > 5000
    sc = scoring_for(path)
    out, recs, edits, dig, cands, ctr = ol.dp_align(sc, case.reads, case.quals, case.refs, case.inp)
    bad = g.compare_dp(case, out, recs, edits, dig, cands)
    assert not bad, "\n".join(bad)
    # the golden set exercises successes, failures, gaps, Ns and multiple calls
    assert (out["status"] == 1).sum() > 1000 and (out["status"] == 0).sum() > 100
    assert (recs["gaps"] > 0).sum() > 100 and (recs["ns"] > 0).sum() > 10
    assert (out["nrec"] > 1).sum() > 100


@pytest.mark.parametrize("gold", I16_DP_SETS)
def test_dp_i16_matches_reference(gold):
    """The oracle's i16 mode (BT2X_DP_I16: int16 cells shifted by 0x8000, no clamp of minsc,
    the i16 reseed) vs alignEnd2EndSseI16 / backtraceNucleotidesEnd2EndSseI16 and the i16
    nextAlignment (aligner_swsse_ee_i16.cpp, aligner_sw.cpp:338-348): statuses, bests (the
    reference's lrmax - 0xff of the int16), E/F/H digests of the int16 cells, candidates,
    every record and the RNG state after every call."""
    path = os.path.join(g.GOLDEN, gold)
    case = g.DpCase(path)
    sc = scoring_for(path)
    out, recs, edits, dig, cands, ctr = ol.dp_align(sc, case.reads, case.quals, case.refs, case.inp)
    bad = g.compare_dp(case, out, recs, edits, dig, cands)
    assert not bad, "\n".join(bad)
    i16 = (case.inp["flags"] & g.abi.DP_I16) != 0
    assert i16.sum() > 1000 and (out["nrec"] > 1).sum() > 500 and (recs["gaps"] > 0).sum() > 100
    if gold == "dp_rep_i16.txt.xz":
        assert i16.all() and (out["status"] == 0).sum() > 100
        assert (out["best"][out["status"] == 1] > 30000).all()       # lrmax - 0xff of the int16
    else:
        assert (case.inp["minsc"] < -254).sum() > 1000                 # beyond the u8 kernel's range
    if gold == "dp_rep_i16_mix.txt.xz":
        assert 0 < (~i16).sum() and ((case.inp["minsc"] < -254) == i16).all()


def test_dp_i16_differs_from_u8():
    """The same problems through the u8 kernel give other RNG states (the reseed differs):
    the i16 goldens are a distinct parity target."""
    case = g.DpCase(os.path.join(g.GOLDEN, "dp_rep_i16.txt.xz"))
    inp = case.inp.copy()
    inp["flags"] = 0
    out, recs, _, _, _, _ = ol.dp_align(ol.default_scoring(), case.reads, case.quals, case.refs, inp)
    moved = 0
    for i, p in enumerate(case.probs):
        r = recs[int(out["rec_off"][i]): int(out["rec_off"][i]) + int(out["nrec"][i])]
        rnd = g.replay_rng(p["rseed"], [int(x["ntries"]) for x in r], False)
        moved += sum(1 for k, c in enumerate(p["calls"][:len(rnd)]) if rnd[k] != c["rnd"])
    assert moved > 1000


RESOLVE_SETS = [("lambda_virus", "resolve_lambda.txt.xz"), ("rep", "resolve_rep.txt.xz")]


@pytest.mark.parametrize("name,gold", RESOLVE_SETS)
def test_resolve_matches_reference(golden_dir, name, gold):
    """getOffset + joinedToTextOff restatement vs GroupWalk2S / getOffset / joinedToTextOff
    outputs of the reference (seed-range elements and fragment-boundary probes)."""
    base = g.materialize_index(name, str(golden_dir))
    idx = ol.OracleIndex(base, load_offs=True)
    case = g.ResolveCase(os.path.join(g.GOLDEN, gold))
    assert case.n > 5000 and "W" in case.kinds
    for rej in (0, 1):
        out, ctr = ol.resolve(idx, case.rows, case.qlen, rej)
        assert g.compare_resolve(out, case.exp[rej], case.joff) == 0
    assert ctr["n_lf1"] > 0
    # boundary probes: rows holding those joined offsets, via the oracle's own SA
    n = int(idx.desc.len) + 1
    sa, _ = ol.resolve(idx, np.arange(n, dtype=np.uint64), 0)
    isa = np.empty(n, dtype=np.uint64)
    isa[sa["joff"].astype(np.int64)] = np.arange(n, dtype=np.uint64)
    assert sorted(sa["joff"].tolist()) == list(range(n))
    rows = isa[case.j_off.astype(np.int64)]
    for rej in (0, 1):
        for ql in np.unique(case.j_qlen):
            m = case.j_qlen == ql
            out, _ = ol.resolve(idx, rows[m], int(ql), rej)
            exp = {k: v[m] for k, v in case.j_exp[rej].items()}
            assert g.compare_resolve(out, exp, case.j_off[m]) == 0
    if name == "rep":       # multi-fragment index: straddles and rejections are covered
        assert case.j_exp[0]["straddled"].sum() > 10
        assert (case.j_exp[1]["tidx"] == g.abi.NO_TIDX).sum() > 10
    # the '$' suffix row (offset len) lies in no fragment
    out, _ = ol.resolve(idx, [n - 1 if sa["joff"][n - 1] == n - 1 else int(isa[n - 1])], 1)
    assert out["tidx"][0] == g.abi.NO_TIDX
