"""TEST HELPER (tests/ only; moved out of the product package in round 4). Host-side seed instantiation: MultiSeedResults::instantiateSeeds / SeedAligner::
prepareSeed + instantiateSeed (aligner_seed.cpp:321-447) and the per-read round offsets
of bt2_search.cpp:2555-2578, producing the bt2x_seed_in batch the seed kernel consumes.

  seed length   L = min(multiseedLen (22), rdlen)
  interval      per = max(int(1 + 1.15*sqrt(rdlen)), 1)   ("-i S,1,1.15", --sensitive)
  rounds        nrounds = min(nSeedRounds (2), per); round r starts at off = per*r//nrounds
  # seeds       1 + (rdlen - off - L) // per if rdlen - off > L else 1
  fw seed i     starts at depth = i*per + off in patFw
  rc seed i     starts at rdlen - depth - L in patRc
  invalid       any N (code 4) in the seed (InstantiatedSeed::instantiateExact)
Reads of 256 bp or more are never aligned by the reference (uint8_t lengths).
"""
from __future__ import annotations

import numpy as np

from bt2x import abi

SEED_LEN = 22
N_ROUNDS = 2


def interval(rdlen: int, c: float = 1.0, lin: float = float(np.float32(1.15))) -> int:
    return max(int(c + lin * np.sqrt(float(rdlen))), 1)


def round_offsets(rdlen: int) -> list[int]:
    per = interval(rdlen)
    nrounds = min(N_ROUNDS, per)
    offs = []
    for r in range(nrounds):
        off = (per * r) // nrounds
        if off > 0 and SEED_LEN + off > rdlen:
            break
        offs.append(off)
    return offs


def instantiate(read_codes: np.ndarray, fw_off: int, rc_off: int, roundi: int = 0,
                nofw: bool = False, norc: bool = False):
    """Seeds of one read for one round. read_codes: codes 0-4 of the read as sequenced;
    fw_off / rc_off: offsets of patFw / patRc in the reads buffer.
    Returns list of (fw, seedoffidx, bt2x_seed_in tuple)."""
    rdlen = len(read_codes)
    if rdlen < 1 or rdlen >= 256:
        return []
    offs = round_offsets(rdlen)
    if roundi >= len(offs):
        return []
    off = offs[roundi]
    per = interval(rdlen)
    L = min(SEED_LEN, rdlen)
    nseeds = 1 + (rdlen - off - L) // per if rdlen - off > L else 1
    rc = np.where(read_codes < 4, 3 - read_codes, 4)[::-1]
    out = []
    for fw in (True, False):
        if (fw and nofw) or (not fw and norc):
            continue
        seq = read_codes if fw else rc
        for i in range(nseeds):
            depth = i * per + off
            start = depth if fw else rdlen - depth - L
            if (seq[start:start + L] > 3).any():
                continue
            out.append((fw, i, ((fw_off if fw else rc_off), start, L, (0,) * 6)))
    return out


def batch_fixed_length(reads: np.ndarray, roundi: int = 0):
    """Vectorised instantiation for a (n, rdlen) matrix of equal-length reads.
    Returns (reads_buffer, seed_in, read_index) with patFw and patRc of read k at
    offsets 2*k*rdlen and (2*k+1)*rdlen of reads_buffer."""
    n, rdlen = reads.shape
    rc = np.where(reads < 4, 3 - reads, 4).astype(np.uint8)[:, ::-1]
    buf = np.ascontiguousarray(np.stack([reads, rc], axis=1).reshape(-1))
    offs = round_offsets(rdlen)
    if roundi >= len(offs):
        return buf, np.zeros(0, dtype=abi.SEED_IN), np.zeros(0, dtype=np.int64)
    off = offs[roundi]
    per = interval(rdlen)
    L = min(SEED_LEN, rdlen)
    nseeds = 1 + (rdlen - off - L) // per if rdlen - off > L else 1
    depth = np.arange(nseeds) * per + off
    starts = np.concatenate([depth, rdlen - depth - L])            # fw seeds then rc seeds
    strand = np.concatenate([np.zeros(nseeds, np.int64), np.ones(nseeds, np.int64)])
    ridx = np.repeat(np.arange(n), 2 * nseeds)
    st = np.tile(starts, n)
    sd = np.tile(strand, n)
    src = np.where(sd[:, None] == 0, reads[ridx], rc[ridx])
    win = np.take_along_axis(src, st[:, None] + np.arange(L)[None, :], axis=1)
    valid = (win <= 3).all(axis=1)
    sin = np.zeros(int(valid.sum()), dtype=abi.SEED_IN)
    sin["read_off"] = ((2 * ridx + sd) * rdlen)[valid]
    sin["seed_off"] = st[valid]
    sin["seed_len"] = L
    return buf, sin, ridx[valid]
