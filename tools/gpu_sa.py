"""Suffix array of a joined reference text by prefix doubling on the GPU (torch sorts).

Bench-input tooling, not the measured path: it lets bench.py index a genome-scale
synthetic reference on the GPU box in seconds, then bt2x_build_index_sa writes the
.bt2l files from it (byte-identical to bt2x_build_index / the reference's builder,
tests/test_builder.py).  Order is the reference's: '$' (end of text) sorts after every
base, so shorter suffixes sort after longer ones that share their prefix
(Ebwt::buildToDisk's SA, bt2_idx.h:2922).

Round 0 sorts 21-character keys (3 bits/char: A,C,G,T = 0..3, '$' = 4); round k
sorts (rank[i], rank[i + h]) pairs packed into one int64: (rank[i] - 2^31) << 32 |
rank[i + h], order-preserving for dense ranks < n+1 <= 2^32 (hg38-scale texts), h
doubling from 21 until every rank is unique.
"""
from __future__ import annotations

import numpy as np


# torch.sort and torch.cumsum take at most INT_MAX elements along a dimension; hg38-scale
# texts (3.1 G suffixes) are sorted as value-range buckets and scanned in chunks.
_LIMIT = (1 << 31) - 1
_CHUNK = 1 << 30


def _cumsum(x, dtype):
    import torch
    if x.numel() <= _LIMIT:
        return torch.cumsum(x, 0, dtype=dtype)
    out = torch.empty(x.numel(), dtype=dtype, device=x.device)
    carry = 0
    for c0 in range(0, x.numel(), _CHUNK):
        seg = torch.cumsum(x[c0:c0 + _CHUNK], 0, dtype=dtype)
        seg += carry
        carry = int(seg[-1])
        out[c0:c0 + seg.numel()] = seg
    return out


def _sort(key):
    """(sorted values, permutation) of a 1-D int64 tensor of any length: below INT_MAX one
    torch.sort; above, buckets of key ranges (splitters from a sorted sample; equal keys
    share a bucket), each gathered chunk by chunk and sorted on its own."""
    import torch
    n = key.numel()
    if n <= _LIMIT:
        return torch.sort(key)
    nb = -(-n // (_LIMIT // 2))
    samp = torch.sort(key[torch.randint(0, n, (min(n, 1 << 22),), device=key.device)]).values
    splits = [int(samp[(len(samp) * k) // nb]) for k in range(1, nb)]
    vals, perm = [], []
    for b in range(nb):
        pv, pi = [], []
        for c0 in range(0, n, _CHUNK):
            kc = key[c0:c0 + _CHUNK]
            m = torch.ones_like(kc, dtype=torch.bool)
            if b > 0:
                m &= kc >= splits[b - 1]
            if b < nb - 1:
                m &= kc < splits[b]
            pv.append(kc[m])
            pi.append(torch.nonzero(m).squeeze(1) + c0)
            del m
        v = torch.cat(pv)
        i = torch.cat(pi)
        del pv, pi
        if v.numel() > _LIMIT:
            raise RuntimeError("gpu_sa: a key bucket exceeds INT_MAX elements")
        sv, sp = torch.sort(v)
        vals.append(sv)
        perm.append(i[sp])
        del v, i, sv, sp
    return torch.cat(vals), torch.cat(perm)


def suffix_array(codes: np.ndarray, device="cuda", max_rounds: int = 40, ftab_chars: int = 10):
    """codes: uint8 joined text (values 0..3).  Returns (sa, bwt, keys): uint64 SA of
    length len+1 plus the per-row gathers bt2x_build_index_sa accepts (bwt[i] =
    text[sa[i]-1], keys[i] = ftab_chars-mer at sa[i])."""
    import torch
    n = len(codes)
    N = n + 1
    if N >= (1 << 32):
        raise ValueError("gpu_sa: text too long for 32-bit ranks")
    dev = torch.device(device)
    t = torch.zeros(N + 21, dtype=torch.int64, device=dev)
    t[:n] = torch.from_numpy(np.ascontiguousarray(codes)).to(dev)
    t[n] = 4
    key = torch.zeros(N, dtype=torch.int64, device=dev)
    for k in range(21):
        key.bitwise_left_shift_(3).bitwise_or_(t[k:k + N])
    del t
    h = 21
    rank = None
    for _ in range(max_rounds):
        vals, sa = _sort(key)
        del key
        head = torch.ones(N, dtype=torch.int32, device=dev)
        head[1:] = (vals[1:] != vals[:-1]).to(torch.int32)
        del vals
        done = bool(head.all())
        # dense rank of each sorted suffix's group (cumsum, not cummax: far faster on ROCm)
        gid = _cumsum(head, torch.int64)
        gid -= 1
        del head
        rank = torch.empty(N, dtype=torch.int64, device=dev)
        rank[sa] = gid
        del gid
        if done:
            del rank
            return _finish(codes, sa, dev, ftab_chars)
        del sa
        key = (rank - (1 << 31)).mul_(1 << 32)
        key[: N - h] += rank[h:]
        del rank
        h *= 2
    raise RuntimeError("gpu_sa: prefix doubling did not converge")


def _finish(codes, sa, dev, ftab_chars):
    import torch
    n = len(codes)
    c = torch.from_numpy(np.ascontiguousarray(codes)).to(dev)
    bwt = c[(sa - 1).clamp_(min=0)]
    km = torch.zeros(n + 1, dtype=torch.int32, device=dev)
    m = n - ftab_chars + 1
    if m > 0:
        for k in range(ftab_chars):
            km[:m].bitwise_left_shift_(2).bitwise_or_(c[k:k + m].to(torch.int32))
    keys = km[sa]
    return (sa.cpu().numpy().view(np.uint64), bwt.cpu().numpy(),
            keys.cpu().numpy().view(np.uint32))
