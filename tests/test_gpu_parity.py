"""Parity of the gfx950 kernels (through the C-ABI, libbt2x.so) with the reference's
golden vectors and with the CPU oracle.  Integer/byte/index work: bit-exact."""
import os

import numpy as np
import pytest

import golden_io as g
import oracle_lib as ol
from bt2x import abi, lib  # noqa: E402
import framing_ref as framing  # noqa: E402

pytestmark = pytest.mark.gpu

SEED_SETS = [("lambda_virus", "lambda_longreads.fq.xz", "seeds_lambda.txt.xz"),
             ("rep", "rep_reads.fq.xz", "seeds_rep.txt.xz")]
DP_SETS = ["dp_rep.txt.xz", "dp_rep_dpad12.txt.xz", "dp_rep_alt.txt.xz",
           # the reference's i16 kernel (-DENABLE_I16 build): --no-sse8, minimum scores below
           # the u8 floor, and that build's default (mixed u8/i16 launches)
           "dp_rep_i16.txt.xz", "dp_rep_i16_wide.txt.xz", "dp_rep_i16_mix.txt.xz"]


@pytest.fixture(scope="module")
def ctxs(golden_dir):
    out = {}
    for name in ("lambda_virus", "rep"):
        base = g.materialize_index(name, str(golden_dir))
        idx = lib.Index(base, load_offs=True)            # SA sample + text: full SA in HBM
        out[name] = (lib.Context(idx), ol.OracleIndex(base))
    return out


@pytest.mark.parametrize("name,fq,gold", SEED_SETS)
def test_seed_kernel_matches_reference_golden(ctxs, name, fq, gold):
    ctx, _ = ctxs[name]
    case = g.SeedCase(os.path.join(g.GOLDEN, fq), os.path.join(g.GOLDEN, gold))
    out = ctx.seed_search(case.reads, case.inp, do_extend=True)
    np.testing.assert_array_equal(out["need_reporting"], case.exp_rep)
    np.testing.assert_array_equal(out["topf"], case.exp_topf)
    np.testing.assert_array_equal(out["botf"], case.exp_botf)
    np.testing.assert_array_equal(out["nlex"], case.exp_nlex)
    ms = ctx.last_kernel_ms(abi.K_SEED)
    assert ms > 0
    c = ctx.last_counters(abi.K_SEED)
    _, oc = ol.seed_search(ctxs[name][1], case.reads, case.inp)
    assert (c["n_bilf"], c["n_lf1"], c["n_ftab"]) == (oc["n_bilf"], oc["n_lf1"], oc["n_ftab"])


def test_seed_kernel_without_extension(ctxs):
    ctx, oidx = ctxs["rep"]
    case = g.SeedCase(os.path.join(g.GOLDEN, "rep_reads.fq.xz"), os.path.join(g.GOLDEN, "seeds_rep.txt.xz"))
    out = ctx.seed_search(case.reads, case.inp, do_extend=False)
    exp, _ = ol.seed_search(oidx, case.reads, case.inp, do_extend=False)
    np.testing.assert_array_equal(out, exp)
    assert (out["nlex"] == 0).all()


def scoring_pair(path):
    kv = g.dp_header_scoring(path)
    return lib.default_scoring(**kv), kv


@pytest.mark.parametrize("gold", DP_SETS)
def test_dp_kernel_matches_reference_golden(ctxs, gold):
    path = os.path.join(g.GOLDEN, gold)
    case = g.DpCase(path)
    sc, kv = scoring_pair(path)
    ctx = lib.Context(ctxs["rep"][0].index, scoring=sc)
    out, recs, edits, dig, cands = ctx.dp_align(case.reads, case.quals, case.refs, case.inp, debug=True)
    bad = g.compare_dp(case, out, recs, edits, dig, cands)
    assert not bad, "\n".join(bad)
    c = ctx.last_counters(abi.K_DP)
    assert c["dp_cells"] == int((case.inp["rdlen"].astype(np.int64) * case.inp["ncol"]).sum())
    ctx.close()


def test_dp_kernel_matches_oracle_at_scale(ctxs):
    """40k framed problems on the repeat-rich genome, incl. shifted diagonals, N-rich reads
    and both strands: HIP vs the C oracle, every output field."""
    import lzma
    import simdata as sd
    with lzma.open(os.path.join(g.GOLDEN, "rep.fa.xz"), "rb") as f:
        tmp = f.read()
    chroms, cur, name = [], [], None
    for line in tmp.split(b"\n"):
        if line.startswith(b">"):
            if name is not None:
                chroms.append((name, b"".join(cur)))
            name, cur = line[1:].decode(), []
        elif line:
            cur.append(line)
    chroms.append((name, b"".join(cur)))
    ref = [g.codes(s) for _, s in chroms]
    reads = (sd.sim_reads(chroms, 16000, 100, seed=101) + sd.sim_reads(chroms, 8000, 139, seed=102)
             + sd.sim_reads(chroms, 4000, 60, seed=103, n_rate=0.05, sub_rate=0.05)
             + sd.sim_reads(chroms, 4000, 30, seed=104))
    rng = np.random.default_rng(5)
    tidx, off, fw, rc, qc = [], [], [], [], []
    for nm, s, q in reads:
        _, c, o, f = nm.split(":")
        shift = int(rng.choice([0, 0, 1, -1, 3, -7, 15]))
        tidx.append(int(c)); off.append(int(o) + shift); fw.append(bool(int(f)) ^ (rng.random() < 0.1))
        rc.append(g.codes(s)); qc.append(np.frombuffer(q, np.uint8))
    # framing takes the read as sequenced; for rc-strand reads the oriented read is patRc
    rd, qu, rf, dp, keep = framing.build_dp_batch(ref, tidx, off, fw, rc, qc)
    assert keep.sum() > 30000
    ctx = ctxs["rep"][0]
    out, recs, edits, dig, cands = ctx.dp_align(rd, qu, rf, dp, debug=True)
    sc = ol.default_scoring()
    eo, erecs, eedits, edig, ecands, _ = ol.dp_align(sc, rd, qu, rf, dp)
    np.testing.assert_array_equal(out[["status", "best", "ncand", "nrec"]], eo[["status", "best", "ncand", "nrec"]])
    np.testing.assert_array_equal(dig, edig)
    np.testing.assert_array_equal(cands, ecands)
    # records: compare per problem (arena order differs)
    for i in np.nonzero(out["nrec"])[0]:
        a = recs[out["rec_off"][i]: out["rec_off"][i] + out["nrec"][i]]
        b = erecs[eo["rec_off"][i]: eo["rec_off"][i] + eo["nrec"][i]]
        fields = ["ntries", "ok", "score", "ns", "gaps", "nedit", "bases_aligned", "refns", "refoff", "nbuf"]
        assert (a[fields] == b[fields]).all(), i
        for ra, rb in zip(a, b):
            # the edit-buffer image (bt2x.h): the alignment's edits are its prefix
            np.testing.assert_array_equal(edits[ra["edit_off"]: ra["edit_off"] + ra["nbuf"]],
                                          eedits[rb["edit_off"]: rb["edit_off"] + rb["nbuf"]])
    assert (out["status"] == 1).sum() > 20000
    assert (recs["nbuf"] > recs["nedit"]).sum() > 1000      # failed attempts' leftovers are exercised

    # the same problems naming their windows (BT2X_DP_REF_TEXT: cut on the GPU from the
    # resident joined text through the fragment table, N runs included): identical results
    assert ctx.capabilities() & abi.CAP_REF_TEXT
    dp2 = dp.copy()
    dp2["ref_off"] = np.asarray(tidx, dtype=np.uint64)[np.nonzero(keep)[0]]
    dp2["flags"] |= abi.DP_REF_TEXT
    assert any((c == 4).any() for c in ref)                  # the fixture's N runs reach windows
    out2, recs2, edits2, dig2, cands2 = ctx.dp_align(rd, qu, rf, dp2, debug=True)
    np.testing.assert_array_equal(out2[["status", "best", "ncand", "nrec"]], eo[["status", "best", "ncand", "nrec"]])
    np.testing.assert_array_equal(dig2, edig)
    np.testing.assert_array_equal(cands2, ecands)
    o3, r3, e3 = ctx.dp_align(rd, qu, np.zeros(0, np.uint8), dp2, debug=False)[:3]   # no refs at all
    _compare_out(o3, eo, dp)

    # the production kernels without debug outputs: lane-per-problem and wave-per-problem
    # (the small-launch mode), every record and the whole edit-buffer image
    sel = np.arange(len(dp)) < 12000
    fields = ["ntries", "ok", "score", "ns", "gaps", "nedit", "bases_aligned", "refns", "refoff", "nbuf"]
    # (and every successful walk handed to the wave kernel's parallel walk; the wave mode
    # with the parallel walk)
    # (the u8 lane launches: the two-lanes-per-problem fill, dp_duo_kernel, below 65,536
    # problems; BT2X_DP_DUO=0 the one-lane dp_fill_kernel; BT2X_DP_SPLIT=1 the two-wave
    # split fill, dp_split_kernel)
    # (the wave kernel: its banded layout, whole rectangles, every problem with a candidate
    # or none handed to the wave-parallel walk; the lane kernel's hand-over pass with whole
    # rectangles)
    for wave, env in (("0", {}), ("1", {}), ("1", {"BT2X_DP_WAVE_BAND": "0"}), ("1", {"BT2X_DP_WAVE_HAND": "1"}),
                      ("1", {"BT2X_DP_WAVE_HAND": "0"}), ("0", {"BT2X_DP_HEAVY": "1", "BT2X_DP_WAVE_BAND": "0"}),
                      ("0", {"BT2X_DP_HEAVY": "1"}), ("1", {"BT2X_DP_PARWALK": "2"}),
                      ("0", {"BT2X_DP_SPLIT": "1"}), ("0", {"BT2X_DP_SPLIT": "1", "BT2X_DP_HEAVY": "1"}),
                      ("0", {"BT2X_DP_DUO": "0"}),
                      ("0", {"BT2X_DP_DUO": "0", "BT2X_DP_HEAVY": "1"})):
        os.environ["BT2X_DP_WAVE"] = wave
        os.environ.update(env)
        try:
            out, recs, edits = ctx.dp_align(rd, qu, rf, dp, debug=False)[:3]
        finally:
            del os.environ["BT2X_DP_WAVE"]
            for k in env:
                del os.environ[k]
        _compare_out(out, eo, dp)
        for i in np.nonzero(out["nrec"] * sel)[0]:
            a = recs[out["rec_off"][i]: out["rec_off"][i] + out["nrec"][i]]
            b = erecs[eo["rec_off"][i]: eo["rec_off"][i] + eo["nrec"][i]]
            assert (a[fields] == b[fields]).all(), (wave, i)
            for ra, rb in zip(a, b):
                np.testing.assert_array_equal(edits[ra["edit_off"]: ra["edit_off"] + ra["nbuf"]],
                                              eedits[rb["edit_off"]: rb["edit_off"] + rb["nbuf"]])


def test_dp_rejects_shapes_outside_reference_limits(ctxs):
    ctx = ctxs["rep"][0]
    dp = np.zeros(1, dtype=abi.DP_IN)
    dp["rdlen"], dp["ncol"], dp["minsc"] = 161, 100, -60           # > ALN_MAX_ROWS
    z = np.zeros(400, np.uint8)
    with pytest.raises(lib.Bt2xError):
        ctx.dp_align(z, z + 40, z, dp)
    dp["rdlen"], dp["ncol"] = 100, 200                               # ncol+1 > ALN_MAX_COLS
    with pytest.raises(lib.Bt2xError):
        ctx.dp_align(z, z + 40, z, dp)


SHIM = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "test_shims")


def _golden_records(gold):
    """Per problem: (P fields, [A line tokens], [N lines]) straight from the golden text."""
    out = []
    with g.open_text(os.path.join(g.GOLDEN, gold)) as f:
        for line in f:
            t = line.split()
            if not t:
                continue
            if t[0] == "P":
                out.append((t, None, []))
            elif t[0] == "A":
                out[-1] = (out[-1][0], t, out[-1][2])
            elif t[0] == "N":
                out[-1][2].append(line.strip())
    return out


@pytest.mark.parametrize("gold,mode,limit", [("dp_rep.txt.xz", "batch", None),
                                             ("dp_rep_alt.txt.xz", "batch", None),
                                             ("dp_rep_dpad12.txt.xz", "single", 400),
                                             ("dp_rep_i16.txt.xz", "batch", None),
                                             ("dp_rep_i16_mix.txt.xz", "batch", None),
                                             ("dp_rep_i16_wide.txt.xz", "single", 300)])
def test_cpp_host_shims_match_golden(golden_dir, tmp_path, gold, mode, limit):
    """include/bt2x_shims.hpp driven like SwDriver drives SwAligner (initRead, initRef,
    align, nextAlignment until done, the caller's RandomSource advanced by the shim)
    reproduces the reference's records line for line.  The i16 goldens run the shims as a
    -DENABLE_I16 build compiles them (tests/cpp/test_shims_i16), with the golden's sse8."""
    import subprocess
    shim = SHIM + ("_i16" if "_i16" in gold else "")
    assert os.access(shim, os.X_OK), f"{shim} not built (__graft_entry__.build())"
    recs = _golden_records(gold)[:limit]
    pf = tmp_path / "probs.txt"
    with open(pf, "w") as f:
        for t, _, _ in recs:
            # fw seq qual win refl refr triml corel corer minsc nceil rseed tlen
            f.write(" ".join([t[3], t[4], t[5], t[6], t[7], t[8], t[9], t[10], t[11], t[12], t[13],
                              t[14], t[17]]) + "\n")
    s = g.dp_header_scoring(os.path.join(g.GOLDEN, gold))
    args = [str(s[k]) for k in ("gapbar", "mm_max", "mm_min", "n_pen", "rdg_const", "rdg_linear",
                                "rfg_const", "rfg_linear")] + [str(g.dp_header_sse8(os.path.join(g.GOLDEN, gold)))]
    base = g.materialize_index("rep", str(golden_dir))
    r = subprocess.run([shim, base, str(pf), mode] + args, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    got = {}
    cur = None
    for line in r.stdout.splitlines():
        t = line.split()
        if t[0] == "P":
            cur = int(t[1])
            got[cur] = (None, [])
        elif t[0] == "A":
            got[cur] = (t, got[cur][1])
        elif t[0] == "N":
            got[cur][1].append(line.strip())
    assert len(got) == len(recs)
    ncalls = 0
    for i, (_, a, ns) in enumerate(recs):
        ga, gn = got[i]
        k = 4 if mode == "batch" else 3
        # align()'s verdict, best (exact for failed problems too: BT2X_OPT_EXACT_BEST) and
        # candidate count, then every nextAlignment call
        assert ga[:k] == a[:k], (i, ga, a)
        assert gn == ns, (i, gn, ns)
        ncalls += len(ns)
    assert ncalls > 0


@pytest.mark.parametrize("name,fasta", [("lambda_virus", "lambda_virus.fa"), ("rep", "rep.fa.xz")])
def test_device_full_suffix_array(ctxs, tmp_path, name, fasta):
    """The suffix array rebuilt in HBM from the SA sample (LF walks from sampled rows)
    equals the suffix array of the joined text (tools/gpu_sa.py on the CPU)."""
    import lzma
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(g.HERE), "tools"))
    import gpu_sa
    import simdata as sd
    src = os.path.join(g.GOLDEN, fasta)
    fa = str(tmp_path / "in.fa")
    with (lzma.open(src, "rb") if src.endswith(".xz") else open(src, "rb")) as fi, open(fa, "wb") as fo:
        fo.write(fi.read())
    codes, _ = sd.concat_genome(sd.read_fasta(fa))
    sa, _, _ = gpu_sa.suffix_array(codes[codes < 4], device="cpu")
    ctx = ctxs[name][0]
    got = ctx.suffix_array()
    np.testing.assert_array_equal(got, sa.astype(np.uint32))


def test_seed_kernel_lf_extension_path(golden_dir, monkeypatch):
    """Without the full SA (BT2X_FULL_SA=0) unique-range extension runs as LF walks;
    same results against the reference golden."""
    monkeypatch.setenv("BT2X_FULL_SA", "0")
    base = g.materialize_index("rep", str(golden_dir))
    ctx = lib.Context(lib.Index(base, load_offs=True))
    case = g.SeedCase(os.path.join(g.GOLDEN, "rep_reads.fq.xz"), os.path.join(g.GOLDEN, "seeds_rep.txt.xz"))
    out = ctx.seed_search(case.reads, case.inp, do_extend=True)
    np.testing.assert_array_equal(out["topf"], case.exp_topf)
    np.testing.assert_array_equal(out["botf"], case.exp_botf)
    np.testing.assert_array_equal(out["nlex"], case.exp_nlex)
    np.testing.assert_array_equal(out["need_reporting"], case.exp_rep)
    with pytest.raises(lib.Bt2xError):
        ctx.suffix_array(0, 1)


def _random_dp_problems(n, seed, i16=0.0):
    """Unframed DP problems over the ABI's whole shape range: R 1..160, ncol 1..199
    (ncol + 1 <= 200), minsc -254..0, random core diagonals / trims, both strands, N-rich
    reads and windows, every quality; lengths mixed within waves.  A fraction `i16` are
    BT2X_DP_I16 problems, half of them with minimum scores below the u8 floor (to -1500)."""
    rng = np.random.default_rng(seed)
    R = rng.integers(1, 161, size=n)
    R[rng.random(n) < 0.1] = 160
    C = rng.integers(1, 200, size=n)
    C[rng.random(n) < 0.1] = 199
    rd, qu, rf = [], [], []
    inp = np.zeros(n, dtype=abi.DP_IN)
    pr = pf = 0
    for i in range(n):
        r, c = int(R[i]), int(C[i])
        ref = rng.integers(0, 4, size=c).astype(np.uint8)
        ref[rng.random(c) < rng.choice([0.0, 0.02, 0.3])] = 4
        # reads: a mutated copy of a window slice (so alignments exist) or random
        st = int(rng.integers(0, max(1, c - r + 1)))
        read = np.resize(ref[st:st + r], r).copy() if rng.random() < 0.7 else rng.integers(0, 4, r).astype(np.uint8)
        read[read > 3] = rng.integers(0, 4)
        mut = rng.random(r) < rng.choice([0.0, 0.02, 0.1])
        read[mut] = rng.integers(0, 5, size=int(mut.sum()))
        q = rng.integers(33, 33 + 42, size=r).astype(np.uint8)
        rd.append(read); qu.append(q); rf.append(ref)
        x = inp[i]
        x["read_off"], x["qual_off"], x["ref_off"] = pr, pr, pf
        x["refl"] = int(rng.integers(-50, 10**6))
        x["rdlen"], x["ncol"] = r, c
        x["minsc"] = int(rng.choice([0, -1, -30, -90, -150, -254, int(rng.integers(-254, 1))]))
        x["nceil"] = int(rng.integers(0, r + 1))
        x["triml"] = int(rng.integers(0, 20))
        lo = int(rng.integers(0, c + 20))
        x["corel"], x["corer"] = lo, lo + int(rng.integers(0, 40))
        x["fw"] = int(rng.random() < 0.5)
        if rng.random() < i16:
            x["flags"] = abi.DP_I16
            if rng.random() < 0.5:
                x["minsc"] = int(rng.integers(-1500, -254))
        pr += r; pf += c
    return np.concatenate(rd), np.concatenate(qu), np.concatenate(rf), inp


def _compare_out(out, eo, inp, exact_best=True):
    """align() verdicts, bit-exact.  Without BT2X_OPT_EXACT_BEST the banded production fill
    (dp_kernel.hip, BT2X_DP_BAND) computes only cells a path scoring >= minsc can use, so
    `best` of a failed problem may come out lower than the reference's, still below the
    reference's threshold (u8: minsc; i16: the reference's own lrmax - 0xff test)."""
    np.testing.assert_array_equal(out[["status", "ncand", "nrec"]], eo[["status", "ncand", "nrec"]])
    if exact_best:
        np.testing.assert_array_equal(out["best"], eo["best"])
        return
    ok = eo["status"] == 1
    np.testing.assert_array_equal(out["best"][ok], eo["best"][ok])
    assert (out["best"][~ok] <= eo["best"][~ok]).all()


def _compare_dp(out, recs, edits, eo, erecs, eedits, inp, exact_best=True):
    _compare_out(out, eo, inp, exact_best)
    fields = ["ntries", "ok", "score", "ns", "gaps", "nedit", "bases_aligned", "refns", "refoff"]
    for i in np.nonzero(out["nrec"])[0]:
        a = recs[out["rec_off"][i]: out["rec_off"][i] + out["nrec"][i]]
        b = erecs[eo["rec_off"][i]: eo["rec_off"][i] + eo["nrec"][i]]
        assert (a[fields] == b[fields]).all(), i
        for ra, rb in zip(a, b):
            np.testing.assert_array_equal(edits[ra["edit_off"]: ra["edit_off"] + ra["nedit"]],
                                          eedits[rb["edit_off"]: rb["edit_off"] + rb["nedit"]])


@pytest.mark.parametrize("debug,wave,band,i16,heavy,parwalk,duo", [
    (False, "0", "1", 0.0, None, None, None), (False, "0", "0", 0.0, None, None, None),
    (False, "1", "1", 0.0, None, None, None), (True, "0", "1", 0.0, None, None, None),
    (False, "0", "1", 1.0, None, None, None), (False, "1", "1", 1.0, None, None, None),
    (True, "0", "1", 1.0, None, None, None), (False, "0", "1", 0.3, None, None, None),
    (True, "0", "1", 0.3, None, None, None),
    (False, "0", "1", 0.0, "0", None, None), (False, "0", "1", 0.0, "1", None, None),
    (False, "0", "1", 0.3, "1", None, None), (False, "0", "0", 1.0, "2", None, None),
    (False, "0", "1", 0.0, "1", "0", None), (False, "1", "1", 0.0, None, "2", None), (False, "1", "1", 1.0, None, "2", None),
    (False, "1", "1", 0.3, None, "2", None),
    (False, "0", "1", 0.0, None, None, "0"), (False, "0", "1", 0.0, "0", None, "0"), (False, "0", "1", 0.0, "1", None, "0"),
    (False, "0", "1", 0.0, None, None, "split"), (False, "0", "1", 0.0, "1", None, "split"),
    (False, "0", "1", 0.0, "2", None, None),
    (False, "1f", "1", 0.0, None, None, None), (False, "1f", "1", 1.0, None, None, None),
    (False, "1f", "1", 0.3, None, "2", None), (False, "1", "1", 0.3, "0", None, None),
    (False, "0f", "1", 0.3, "1", None, None)])
def test_dp_kernel_edge_shapes_vs_oracle(ctxs, debug, wave, band, i16, heavy, parwalk, duo, monkeypatch):
    """Production (debug=False; lane-per-problem kernel with and without the diagonal band,
    wave-per-problem mode) and debug kernels on random shapes/penalty thresholds at the ABI
    limits vs the oracle: statuses, bests, candidates, every nextAlignment record and edit.
    i16: the share of BT2X_DP_I16 problems (all, or mixed into u8 launches; the 16-bit lane
    kernels, including minimum scores below -254).  heavy: BT2X_DP_HEAVY, the walk-step budget
    past which the lane kernel drops a problem for the wave kernel to redo (0: never; 1 and 2:
    nearly every successful problem, mid-walk; default 800).  parwalk: BT2X_DP_PARWALK, the
    wave kernel's nextAlignment sequence on all lanes (walk_wave_par; default: for the walks
    handed over, 2: the small-launch mode too, 0: lane 0 everywhere).  duo: the banded u8
    lane launches' fill -- None: the launcher's default (dp_duo_kernel at these sizes);
    "1" / "0": BT2X_DP_DUO, two lanes per problem (dp_duo_kernel) or one (dp_fill_kernel);
    "split": BT2X_DP_SPLIT=1, the two-wave split fill (dp_split_kernel).  wave "1" runs the
    wave kernel with its banded traceback layout (problems whose band window does not fit
    go to the whole-rectangle pass; with heavy "0" there is no hand-over list and the whole
    rectangle is kept), "1f" with whole rectangles in LDS (BT2X_DP_WAVE_BAND=0)."""
    if wave.endswith("f"):
        wave = wave[:-1]
        monkeypatch.setenv("BT2X_DP_WAVE_BAND", "0")
    monkeypatch.setenv("BT2X_DP_WAVE", wave)
    monkeypatch.setenv("BT2X_DP_BAND", band)
    if duo == "split":
        monkeypatch.setenv("BT2X_DP_SPLIT", "1")
    elif duo is not None:
        monkeypatch.setenv("BT2X_DP_DUO", duo)
    if heavy is not None:
        monkeypatch.setenv("BT2X_DP_HEAVY", heavy)
    if parwalk is not None:
        monkeypatch.setenv("BT2X_DP_PARWALK", parwalk)
    rd, qu, rf, inp = _random_dp_problems(6000, seed=77 + int(debug) + int(10 * i16), i16=i16)
    ctx = ctxs["rep"][0]
    res = ctx.dp_align(rd, qu, rf, inp, debug=debug)
    eo, erecs, eedits, edig, ecands, _ = ol.dp_align(ol.default_scoring(), rd, qu, rf, inp)
    out, recs, edits = res[0], res[1], res[2]
    _compare_dp(out, recs, edits, eo, erecs, eedits, inp)
    if debug:
        np.testing.assert_array_equal(res[3], edig)
        np.testing.assert_array_equal(res[4], ecands)
    assert (out["status"] == 1).sum() > 1000 and (out["status"] == 0).sum() > 100
    if i16:
        assert ((inp["flags"] == abi.DP_I16) & (inp["minsc"] < -254) & (out["status"] == 1)).sum() > 100


def test_dp_exact_best_option(ctxs, monkeypatch):
    """BT2X_OPT_EXACT_BEST (default on): failed problems' best equals the reference's; off,
    the banded lane kernel may report a lower one (documented in bt2x.h)."""
    monkeypatch.setenv("BT2X_DP_WAVE", "0")
    rd, qu, rf, inp = _random_dp_problems(3000, seed=5)
    eo, erecs, eedits, _, _, _ = ol.dp_align(ol.default_scoring(), rd, qu, rf, inp)
    ctx = ctxs["rep"][0]
    try:
        ctx.set_option(abi.OPT_EXACT_BEST, 0)
        out, recs, edits = ctx.dp_align(rd, qu, rf, inp)[:3]
        _compare_dp(out, recs, edits, eo, erecs, eedits, inp, exact_best=False)
    finally:
        ctx.set_option(abi.OPT_EXACT_BEST, 1)
    out, recs, edits = ctx.dp_align(rd, qu, rf, inp)[:3]
    _compare_dp(out, recs, edits, eo, erecs, eedits, inp)


@pytest.mark.parametrize("gold", ["dp_rep_dpad12.txt.xz", "dp_rep_i16.txt.xz", "dp_rep_i16_mix.txt.xz"])
@pytest.mark.parametrize("wave,heavy,parwalk,duo", [("0", None, None, None), ("1", None, None, None),
                                                    ("0", "1", None, None), ("1", None, "2", None),
                                                    ("0", "1", "0", None), ("0", None, None, "0"),
                                                    ("0", "1", None, "0"), ("0", None, None, "split"),
                                                    ("1f", None, None, None)])
def test_dp_production_kernel_on_golden(ctxs, wave, heavy, parwalk, duo, gold, monkeypatch):
    """The production (non-debug) kernel, in both modes and with walks handed to the wave
    kernel (its parallel walk, and lane 0's), reproduces the reference records of the golden
    set (oracle-checked, then against the golden itself).  wave "1f": the wave kernel with
    whole rectangles in LDS (BT2X_DP_WAVE_BAND=0; "1" is its banded layout)."""
    if wave.endswith("f"):
        wave = wave[:-1]
        monkeypatch.setenv("BT2X_DP_WAVE_BAND", "0")
    monkeypatch.setenv("BT2X_DP_WAVE", wave)
    if heavy is not None:
        monkeypatch.setenv("BT2X_DP_HEAVY", heavy)
    if parwalk is not None:
        monkeypatch.setenv("BT2X_DP_PARWALK", parwalk)
    if duo == "split":                           # the two-wave split fill
        monkeypatch.setenv("BT2X_DP_SPLIT", "1")
    elif duo is not None:
        monkeypatch.setenv("BT2X_DP_DUO", duo)
    case = g.DpCase(os.path.join(g.GOLDEN, gold))
    ctx = ctxs["rep"][0]
    out, recs, edits = ctx.dp_align(case.reads, case.quals, case.refs, case.inp, debug=False)[:3]
    eo, erecs, eedits, _, _, _ = ol.dp_align(ol.default_scoring(), case.reads, case.quals, case.refs, case.inp)
    _compare_dp(out, recs, edits, eo, erecs, eedits, case.inp)
    bad = g.compare_dp(case, out, recs, edits)
    assert not bad, "\n".join(bad)


def test_dp_from_read_store_matches_uploaded_reads(ctxs):
    """bt2x_store_reads + bt2x_dp_align(reads = quals = NULL): every problem's read put in a
    store slot (half of them as the reverse complement, so their rows come from the slot's
    GPU-derived patRc and reversed qualities) gives the records of the ordinary call."""
    case = g.DpCase(os.path.join(g.GOLDEN, "dp_rep_dpad12.txt.xz"))
    ctx = ctxs["rep"][0]
    ref = ctx.dp_align(case.reads, case.quals, case.refs, case.inp, debug=False)[:3]
    inp = case.inp.copy()
    packed, sin = [], np.zeros(len(inp), dtype=abi.STORE_IN)
    off = 0
    comp = np.array([3, 2, 1, 0, 4], np.uint8)
    for i, p in enumerate(case.inp):
        n = int(p["rdlen"])
        rd = case.reads[int(p["read_off"]):int(p["read_off"]) + n]
        qu = case.quals[int(p["qual_off"]):int(p["qual_off"]) + n]
        rc = i % 2 == 1
        fw, fq = (comp[rd[::-1]], qu[::-1]) if rc else (rd, qu)
        packed += [fw, fq]
        slot = 3 * i + 7                            # sparse slots: the store grows to the largest
        sin[i] = (off, slot, n, 0)
        off += 2 * n
        base = slot * abi.STORE_SLOT_BYTES
        inp[i]["read_off"] = base + (n if rc else 0)
        inp[i]["qual_off"] = base + 2 * n + (n if rc else 0)
    ctx.store_reads(np.concatenate(packed), sin)
    got = ctx.dp_align(None, None, case.refs, inp, debug=False)[:3]
    _compare_dp(*got, *ref, case.inp)                    # (record arena offsets come from atomics)


def _sam_tail_py(r, codes, quals):
    """The record tail bt2x_sam_tails writes (restated from the host driver's formatting of a
    mismatch-only record, host/bt2x_align.cpp cigar_md + finish_read)."""
    R = int(r["rdlen"])
    out = f"{R}M\t*\t0\t0\t" + "".join("ACGTN"[min(int(c), 4)] for c in codes) + "\t" + bytes(quals).decode()
    out += f"\tAS:i:{int(r['as_'])}" + (f"\tXS:i:{int(r['xs'])}" if r["has_xs"] else "") + f"\tXN:i:{int(r['xn'])}"
    n = int(r["nmm"])
    out += f"\tXM:i:{n}\tXO:i:0\tXG:i:0\tNM:i:{n}\tMD:Z:"
    prev, mm_last, first = 0, False, True
    for e in range(n):
        p = int(r["mm_pos"][e])
        if p > prev:
            out += str(p - prev)
            mm_last = first = False
        if mm_last or first:
            out += "0"
        out += chr(int(r["mm_chr"][e]))
        mm_last, first, prev = True, False, p + 1
    if R > prev:
        out += str(R - prev)
    elif mm_last:
        out += "0"
    return (out + "\tYT:Z:UU\tYF:Z:LN\n").encode()


def test_sam_tails_from_read_store(ctxs):
    """bt2x_sam_tails: record tails of aligned reads (either strand, 0-16 mismatches at the
    read's ends and anywhere, lengths 1-256, N codes, optional XS) from store slots equal the
    host driver's formatting; malformed requests are refused."""
    ctx = ctxs["rep"][0]
    rng = np.random.default_rng(11)
    comp = np.array([3, 2, 1, 0, 4], np.uint8)
    n = 3000
    lens = rng.integers(1, 257, n)
    lens[:8] = [1, 9, 10, 99, 100, 150, 255, 256]
    packed, sin, reads, off = [], np.zeros(n, dtype=abi.STORE_IN), [], 0
    for i in range(n):
        L = int(lens[i])
        codes = rng.choice(5, L, p=[0.24, 0.24, 0.24, 0.24, 0.04]).astype(np.uint8)
        quals = rng.integers(33, 75, L).astype(np.uint8)
        packed += [codes, quals]
        sin[i] = (off, 2 * i + 1, L, 0)
        off += 2 * L
        reads.append((codes, quals))
    ctx.store_reads(np.concatenate(packed), sin)
    req = np.zeros(n, dtype=abi.SAM_REQ)
    for i in range(n):
        L = int(lens[i])
        req[i]["slot"], req[i]["rdlen"], req[i]["fw"] = 2 * i + 1, L, i % 2
        k = int(rng.integers(0, min(abi.SAM_MAX_MM, L) + 1))
        pos = np.sort(rng.choice(L, k, replace=False))
        if k and i % 7 == 0:
            pos[0] = 0
        if k and i % 5 == 0:
            pos[-1] = L - 1 if k == 1 or pos[-2] < L - 1 else pos[-1]
        req[i]["nmm"] = k
        req[i]["mm_pos"][:k] = pos
        req[i]["mm_chr"][:k] = rng.choice(np.frombuffer(b"ACGTN", np.uint8), k)
        req[i]["as_"] = -int(rng.integers(0, 300))
        req[i]["has_xs"] = i % 3 == 0
        req[i]["xs"] = -int(rng.integers(0, 300))
        req[i]["xn"] = int(rng.integers(0, 4))
    got = ctx.sam_tails(req)
    for i in range(n):
        codes, quals = reads[i]
        if req[i]["fw"] == 0:
            codes, quals = comp[codes[::-1]], quals[::-1]
        assert got[i] == _sam_tail_py(req[i], codes, quals), i
    # (a slot past every read this context's store has held: earlier tests put reads too)
    for bad in ({"nmm": abi.SAM_MAX_MM + 1}, {"slot": 1 << 24}, {"rdlen": 0}):
        r = req[:4].copy()
        for k, v in bad.items():
            r[1][k] = v
        with pytest.raises(lib.Bt2xError):
            ctx.sam_tails(r)
    r = req[req["nmm"] >= 2][:1].copy()
    r[0]["mm_pos"][1] = r[0]["mm_pos"][0]                # not increasing
    with pytest.raises(lib.Bt2xError):
        ctx.sam_tails(r)


def test_empty_batches(ctxs):
    ctx = ctxs["rep"][0]
    out = ctx.seed_search(np.zeros(16, np.uint8), np.zeros(0, dtype=abi.SEED_IN), do_extend=True)
    assert len(out) == 0
    res = ctx.dp_align(np.zeros(1, np.uint8), np.zeros(1, np.uint8), np.zeros(1, np.uint8),
                       np.zeros(0, dtype=abi.DP_IN), debug=False)
    assert len(res[0]) == 0


RESOLVE_SETS = [("lambda_virus", "resolve_lambda.txt.xz"), ("rep", "resolve_rep.txt.xz")]


def _check_resolve(ctx, oidx, case):
    for rej in (0, 1):
        out = ctx.resolve(case.rows, case.qlen, rej)
        assert g.compare_resolve(out, case.exp[rej], case.joff) == 0
    # boundary probes through the rows that hold those offsets (oracle SA)
    n = int(oidx.desc.len) + 1
    sa, _ = ol.resolve(oidx, np.arange(n, dtype=np.uint64), 0)
    isa = np.empty(n, dtype=np.uint64)
    isa[sa["joff"].astype(np.int64)] = np.arange(n, dtype=np.uint64)
    rows = isa[case.j_off.astype(np.int64)]
    for rej in (0, 1):
        for ql in np.unique(case.j_qlen):
            m = case.j_qlen == ql
            out = ctx.resolve(rows[m], int(ql), rej)
            assert g.compare_resolve(out, {k: v[m] for k, v in case.j_exp[rej].items()}, case.j_off[m]) == 0
    # every row of the index, against the oracle ('$' suffix row included)
    allrows = np.arange(n, dtype=np.uint64)
    out = ctx.resolve(allrows, 22, 0)
    exp, _ = ol.resolve(oidx, allrows, 22, 0)
    np.testing.assert_array_equal(out, exp)


@pytest.mark.parametrize("name,gold", RESOLVE_SETS)
def test_resolve_matches_reference_golden(ctxs, golden_dir, name, gold):
    """SA resolution (resident full SA lookup + joinedToTextOff) vs the reference's
    GroupWalk2S / getOffset / joinedToTextOff outputs and the oracle."""
    ctx, _ = ctxs[name]
    base = g.materialize_index(name, str(golden_dir))
    oidx = ol.OracleIndex(base, load_offs=True)
    case = g.ResolveCase(os.path.join(g.GOLDEN, gold))
    _check_resolve(ctx, oidx, case)
    c = ctx.last_counters(abi.K_RESOLVE)
    assert c["n_lf1"] == 0 and c["n_problems"] == int(oidx.desc.len) + 1
    assert ctx.last_kernel_ms(abi.K_RESOLVE) > 0


@pytest.mark.parametrize("env", [{"BT2X_FULL_SA": "0"}, {"BT2X_FM_SIDES": "1"}])
def test_resolve_lf_walk_paths(golden_dir, monkeypatch, env):
    """Without the full SA the kernel walks LF to the SA sample (blocks, or the .bt2l
    sides): same results, and the LF step count equals the oracle's."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    base = g.materialize_index("rep", str(golden_dir))
    ctx = lib.Context(lib.Index(base, load_offs=True))
    oidx = ol.OracleIndex(base, load_offs=True)
    case = g.ResolveCase(os.path.join(g.GOLDEN, "resolve_rep.txt.xz"))
    _check_resolve(ctx, oidx, case)
    c = ctx.last_counters(abi.K_RESOLVE)
    _, oc = ol.resolve(oidx, np.arange(int(oidx.desc.len) + 1, dtype=np.uint64), 22)
    assert c["n_lf1"] == oc["n_lf1"] > 0


def test_resolve_argument_errors(ctxs, golden_dir):
    ctx, oidx = ctxs["rep"]
    with pytest.raises(lib.Bt2xError):
        ctx.resolve([int(oidx.desc.len) + 1], 22)            # row beyond the BWT
    assert len(ctx.resolve([], 22)) == 0
    base = g.materialize_index("rep", str(golden_dir))
    noffs = lib.Context(lib.Index(base, load_offs=False))    # no SA sample: no resolution
    with pytest.raises(lib.Bt2xError):
        noffs.resolve([0], 22)
