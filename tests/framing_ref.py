"""TEST HELPER (tests/ only; moved out of the product package in round 4). Host-side DP problem framing: the arithmetic SwDriver::extendSeeds performs between a
resolved seed hit and SwAligner::initRef, vectorised with numpy.

  min score       Scoring scoreMin "L,-0.6,-0.6" (bt2_search.cpp:394, simple_func.h:90-112),
                  clamped to [-254, 0] (bt2_search.cpp:2480-2491)
  N ceiling       nCeil "L,0,0.15", min(f(rdlen), rdlen) (bt2_search.cpp:2546)
  max gaps        Scoring::maxReadGaps / maxRefGaps (scoring.cpp:42-98)
  rectangle       DynProgFramer::frameSeedExtensionRect (dp_framer.cpp:81-129),
                  trimToRef_ = !gReportOverhangs = true
  window          SwAligner::initRef (aligner_sw.cpp:117-229): ref[refl .. refr] (+1 extra
                  column that the end-to-end DP never uses), N where the reference has N;
                  rflen + 1 must be <= ALN_MAX_COLS (200) or the DP is not attempted.
"""
from __future__ import annotations

import numpy as np

from bt2x import abi

_F32_C = float(np.float32(-0.6))
_F32_L = float(np.float32(-0.6))
_F32_N = float(np.float32(0.15))


def min_score(rdlen, const=_F32_C, lin=_F32_L):
    """SimpleFunc LINEAR f(x) = C + L*x truncated toward zero, then the u8 clamp."""
    x = np.asarray(rdlen, dtype=np.float64)
    v = np.trunc(const + lin * x).astype(np.int64)
    return np.clip(v, -254, 0)


def n_ceil(rdlen, const=0.0, lin=_F32_N):
    x = np.asarray(rdlen, dtype=np.float64)
    v = np.trunc(const + lin * x).astype(np.int64)
    return np.minimum(v, np.asarray(rdlen, dtype=np.int64))


def max_read_gaps(minsc, rdlen, rdg_const=5, rdg_linear=3):
    """Scoring::maxReadGaps: number of read gaps affordable from a perfect score 0."""
    minsc = np.asarray(minsc, dtype=np.int64)
    op, ex = rdg_const + rdg_linear, rdg_linear
    # sc = 0; first gap costs op, then ex; count gaps while sc >= minsc, minus one
    n = np.where(-op >= minsc, 1 + (-op - minsc) // ex, 0)
    return n.astype(np.int64)


def max_ref_gaps(minsc, rdlen, rfg_const=5, rfg_linear=3):
    return max_read_gaps(minsc, rdlen, rfg_const, rfg_linear)


def frame_rect(off, rdlen, reflen, maxrdgap, maxrfgap, maxhalf):
    """DynProgFramer::frameSeedExtensionRect with trimToRef (no overhang allowed).
    Returns dict of arrays: refl, refr, triml, trimr, corel, corer, maxgap, found."""
    off = np.asarray(off, dtype=np.int64)
    rdlen = np.asarray(rdlen, dtype=np.int64)
    reflen = np.asarray(reflen, dtype=np.int64)
    maxgap = np.minimum(np.maximum(maxrdgap, maxrfgap), maxhalf).astype(np.int64)
    refl = off - 2 * maxgap
    refr = off + (rdlen - 1) + 2 * maxgap
    trimr = np.where(refr >= reflen, refr - (reflen - 1), 0)
    triml = np.where(refl < 0, -refl, 0)
    r = {"refl": refl + triml, "refr": refr - trimr, "triml": triml, "trimr": trimr,
         "corel": maxgap, "corer": 3 * maxgap, "maxgap": maxgap}
    # DPRect::entirelyTrimmed
    r["found"] = (r["refl"] <= r["refr"])
    return r


def build_dp_batch(ref_codes: list[np.ndarray], tidx, off, fw, read_codes: list[np.ndarray],
                   read_quals: list[np.ndarray], maxhalf: int = 15, scoring=None):
    """Frame one DP problem per (tidx, off, fw, read) exactly as extendSeeds would for a
    seed hit implying reference offset `off` for the read's upstream end.

    Returns (reads, quals, refs, dp_in, keep) where keep marks problems that pass the
    reference's initRead/initRef capacity checks (others are not DP problems)."""
    n = len(read_codes)
    rdlen = np.array([len(r) for r in read_codes], dtype=np.int64)
    minsc = min_score(rdlen)
    nceil = n_ceil(rdlen)
    rdg = (5, 3) if scoring is None else (scoring.rdg_const, scoring.rdg_linear)
    rfg = (5, 3) if scoring is None else (scoring.rfg_const, scoring.rfg_linear)
    mrd = max_read_gaps(minsc, rdlen, *rdg)
    mrf = max_ref_gaps(minsc, rdlen, *rfg)
    reflen = np.array([len(ref_codes[t]) for t in tidx], dtype=np.int64)
    rect = frame_rect(off, rdlen, reflen, mrd, mrf, maxhalf)
    ncol = rect["refr"] - rect["refl"] + 1
    keep = rect["found"] & (rdlen <= abi.MAX_ROWS) & (ncol + 1 <= abi.MAX_COLS) & (rdlen >= 1)
    idx = np.nonzero(keep)[0]
    dp = np.zeros(len(idx), dtype=abi.DP_IN)
    rd_parts, q_parts, rf_parts = [], [], []
    pr = pq = pf = 0
    for k, i in enumerate(idx.tolist()):
        c = read_codes[i]
        q = read_quals[i]
        if not fw[i]:
            c = np.where(c < 4, 3 - c, 4).astype(np.uint8)[::-1]
            q = q[::-1]
        w = ref_codes[tidx[i]][rect["refl"][i]: rect["refr"][i] + 1]
        rd_parts.append(c); q_parts.append(q); rf_parts.append(w)
        dp[k] = (pr, pq, pf, rect["refl"][i], len(c), len(w), minsc[i], nceil[i],
                 rect["triml"][i], rect["corel"][i], rect["corer"][i], 1 if fw[i] else 0, 0)
        pr += len(c); pq += len(q); pf += len(w)
    cat = lambda parts: np.ascontiguousarray(np.concatenate(parts)) if parts else np.zeros(1, np.uint8)
    return cat(rd_parts), cat(q_parts), cat(rf_parts), dp, keep


def build_dp_batch_fixed(genome: np.ndarray, chrom_starts: np.ndarray, chrom_lens: np.ndarray,
                         chrom, off, fw, reads: np.ndarray, quals: np.ndarray,
                         maxhalf: int = 15, ref_stride: int = abi.MAX_COLS):
    """Vectorised build_dp_batch for equal-length reads over a concatenated genome.
    Oriented reads/quals are laid out with stride rdlen, windows with stride ref_stride.
    Returns (reads_buf, quals_buf, refs_buf, dp_in, keep)."""
    n, R = reads.shape
    chrom = np.asarray(chrom, dtype=np.int64)
    fw = np.asarray(fw, dtype=bool)
    minsc = min_score(np.full(n, R))
    nceil = n_ceil(np.full(n, R))
    rect = frame_rect(off, np.full(n, R), chrom_lens[chrom], max_read_gaps(minsc, R),
                      max_ref_gaps(minsc, R), maxhalf)
    ncol = rect["refr"] - rect["refl"] + 1
    keep = rect["found"] & (R <= abi.MAX_ROWS) & (ncol + 1 <= abi.MAX_COLS)
    idx = np.nonzero(keep)[0]
    m = len(idx)
    rc = np.where(reads < 4, 3 - reads, 4).astype(np.uint8)[:, ::-1]
    ord_reads = np.where(fw[:, None], reads, rc)[idx]
    ord_quals = np.where(fw[:, None], quals, quals[:, ::-1])[idx]
    gstart = chrom_starts[chrom[idx]] + rect["refl"][idx]
    cols = np.arange(ref_stride)[None, :]
    gi = np.minimum(gstart[:, None] + cols, len(genome) - 1)
    win = np.where(cols < ncol[idx][:, None], genome[gi], 4).astype(np.uint8)
    dp = np.zeros(m, dtype=abi.DP_IN)
    k = np.arange(m, dtype=np.int64)
    dp["read_off"] = k * R
    dp["qual_off"] = k * R
    dp["ref_off"] = k * ref_stride
    dp["refl"] = rect["refl"][idx]
    dp["rdlen"] = R
    dp["ncol"] = ncol[idx]
    dp["minsc"] = minsc[idx]
    dp["nceil"] = nceil[idx]
    dp["triml"] = rect["triml"][idx]
    dp["corel"] = rect["corel"][idx]
    dp["corer"] = rect["corer"][idx]
    dp["fw"] = fw[idx].astype(np.uint8)
    return (np.ascontiguousarray(ord_reads).reshape(-1), np.ascontiguousarray(ord_quals).reshape(-1),
            np.ascontiguousarray(win).reshape(-1), dp, keep)
