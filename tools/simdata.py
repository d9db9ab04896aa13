"""Deterministic synthetic genomes and reads (test and bench inputs).

The reference ships one real genome (lambda, example/reference/lambda_virus.fa) and
no simulator usable offline (its scripts/sim needs Math::Random), so the
synthetic inputs for BASELINE.json's configs are generated here, seeded:

* genome: uniform random ACGT per chromosome, plus (a) interspersed repeat
  families -- a few hundred bp element copied many times with ~2% divergence, which
  gives seed ranges > 1 and multi-hit DP work, (b) low-complexity stretches
  (homopolymers / dinucleotides), (c) N runs, which the index excludes from the
  joined text and the DP pads (aligner_sw.cpp:148-184).
* reads: error model of BASELINE.md ("1 % substitutions, 10 % of reads carry one
  indel, 50 % reverse-complemented, Phred uniform 2-40"), plus a small rate of read
  Ns.  The read name encodes the true origin as ``r<i>:<chrom>:<leftmost offset>:<fw>``.
"""
from __future__ import annotations

import numpy as np

ACGT = np.frombuffer(b"ACGTN", dtype=np.uint8)
_COMP = np.zeros(256, dtype=np.uint8)
for a, b in zip(b"ACGTN", b"TGCAN"):
    _COMP[a] = b


def gen_genome(total_len: int, nchrom: int = 1, seed: int = 0, repeat_frac: float = 0.05,
               repeat_len: int = 300, n_runs_per_mb: float = 2.0,
               lowcomp_per_mb: float = 5.0) -> list[tuple[str, bytes]]:
    rng = np.random.Generator(np.random.PCG64(seed))
    per = total_len // nchrom
    out = []
    fam = [rng.integers(0, 4, size=repeat_len, dtype=np.uint8) for _ in range(8)]
    for c in range(nchrom):
        s = rng.integers(0, 4, size=per, dtype=np.uint8)
        # interspersed repeat copies with ~2% divergence
        ncopies = int(per * repeat_frac / repeat_len)
        if ncopies and per > 4 * repeat_len:
            pos = rng.integers(0, per - repeat_len, size=ncopies)
            which = rng.integers(0, len(fam), size=ncopies)
            for p, w in zip(pos.tolist(), which.tolist()):
                el = fam[w].copy()
                mut = rng.random(repeat_len) < 0.02
                el[mut] = rng.integers(0, 4, size=int(mut.sum()), dtype=np.uint8)
                s[p:p + repeat_len] = el
        # low-complexity stretches
        nlow = int(per / 1e6 * lowcomp_per_mb) + (1 if per >= 20000 else 0)
        for _ in range(nlow):
            ln = int(rng.integers(20, 200))
            p = int(rng.integers(0, max(1, per - ln)))
            unit = rng.integers(0, 4, size=int(rng.integers(1, 3)), dtype=np.uint8)
            s[p:p + ln] = np.resize(unit, ln)
        seq = ACGT[s]
        # N runs (excluded from the joined text by the index builder)
        nn = int(per / 1e6 * n_runs_per_mb) + (1 if per >= 20000 else 0)
        for _ in range(nn):
            ln = int(rng.integers(1, 600))
            p = int(rng.integers(0, max(1, per - ln)))
            seq[p:p + ln] = ord("N")
        out.append((f"chr{c + 1}", seq.tobytes()))
    return out


def gen_tandem_genome(nchrom: int = 4, chrom_len: int = 40000, arrays_per_chrom: int = 12,
                      seed: int = 0, div: float = 0.02):
    """Random chromosomes carrying tandem-repeat arrays (unit 2-40 bp, 200-1500 bp long,
    ~div divergence per base).  A read from an array aligns at several unit shifts inside
    one DP window, so one DP problem yields several alignments and the -M score
    tightening (aligner_sw_driver.cpp:589-619) acts between nextAlignment calls of the
    same problem.  Returns (chroms, arrays) with arrays = [(chrom index, start, end)]."""
    rng = np.random.Generator(np.random.PCG64(seed))
    chroms, arrays = [], []
    for c in range(nchrom):
        s = rng.integers(0, 4, size=chrom_len, dtype=np.uint8)
        slot = chrom_len // arrays_per_chrom
        for a in range(arrays_per_chrom):
            u = int(rng.integers(2, 41))
            ln = int(rng.integers(200, min(1500, slot - 100)))
            p = a * slot + int(rng.integers(0, slot - ln))
            unit = rng.integers(0, 4, size=u, dtype=np.uint8)
            arr = np.resize(unit, ln)
            mut = rng.random(ln) < div
            arr[mut] = rng.integers(0, 4, size=int(mut.sum()), dtype=np.uint8)
            s[p:p + ln] = arr
            arrays.append((c, p, p + ln))
        chroms.append((f"tr{c + 1}", ACGT[s].tobytes()))
    return chroms, arrays


def sim_reads_in(chroms, arrays, n: int, rdlen: int, seed: int, **kw):
    """sim_reads with origins drawn from the given (chrom, start, end) intervals (a read
    may run past an interval's end by up to half its length)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    for i in range(n):
        c, a, b = arrays[int(rng.integers(0, len(arrays)))]
        ref = chroms[c][1]
        lo = max(0, a - rdlen // 4)
        hi = max(lo + 1, min(len(ref) - rdlen - 2, b - rdlen // 2))
        p = int(rng.integers(lo, hi))
        sub = [(chroms[c][0], ref[p:p + rdlen + 2])]
        name, seq, q = sim_reads(sub, 1, rdlen, seed=int(rng.integers(0, 2**31)), **kw)[0]
        fields = name.split(":")
        out.append((f"t{i}:{c}:{p + int(fields[2])}:{fields[3]}", seq, q))
    return out


def write_fasta(path: str, chroms: list[tuple[str, bytes]], width: int = 60) -> None:
    with open(path, "wb") as f:
        for name, seq in chroms:
            f.write(b">" + name.encode() + b"\n")
            for i in range(0, len(seq), width):
                f.write(seq[i:i + width] + b"\n")


def read_fasta(path: str) -> list[tuple[str, bytes]]:
    out, name, cur = [], None, []
    with open(path, "rb") as f:
        for line in f:
            line = line.strip()
            if line.startswith(b">"):
                if name is not None:
                    out.append((name, b"".join(cur)))
                name, cur = line[1:].split()[0].decode(), []
            elif line:
                cur.append(line.upper())
    if name is not None:
        out.append((name, b"".join(cur)))
    return out


def revcomp(s: bytes) -> bytes:
    return _COMP[np.frombuffer(s, dtype=np.uint8)[::-1]].tobytes()


def sim_reads(chroms: list[tuple[str, bytes]], n: int, rdlen: int, seed: int,
              sub_rate: float = 0.01, indel_frac: float = 0.10, rc_frac: float = 0.5,
              qmin: int = 2, qmax: int = 40, n_rate: float = 0.001,
              allow_ref_n: bool = False) -> list[tuple[str, bytes, bytes]]:
    """Return [(name, seq, qual)].  Origins avoid reference N runs unless allowed."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lens = np.array([len(s) for _, s in chroms], dtype=np.int64)
    cum = np.cumsum(lens)
    reads = []
    i = 0
    tries = 0
    while len(reads) < n:
        tries += 1
        g = int(rng.integers(0, int(cum[-1])))
        c = int(np.searchsorted(cum, g, side="right"))
        ref = chroms[c][1]
        if len(ref) < rdlen + 2:
            continue
        p = int(rng.integers(0, len(ref) - rdlen - 1))
        frag = bytearray(ref[p:p + rdlen + 1])
        if not allow_ref_n and b"N" in frag:
            continue
        s = np.frombuffer(bytes(frag[:rdlen]), dtype=np.uint8).copy()
        mut = rng.random(rdlen) < sub_rate
        s[mut] = ACGT[rng.integers(0, 4, size=int(mut.sum()))]
        if rdlen > 24 and rng.random() < indel_frac:
            k = int(rng.integers(10, rdlen - 10))
            if rng.random() < 0.5:      # deletion from the read
                s = np.concatenate([s[:k], s[k + 1:], np.frombuffer(bytes(frag[rdlen:rdlen + 1]), np.uint8)])
            else:                       # insertion into the read
                s = np.concatenate([s[:k], ACGT[rng.integers(0, 4, size=1)], s[k:-1]])
        nm = rng.random(rdlen) < n_rate
        s[nm] = ord("N")
        fw = rng.random() >= rc_frac
        seq = s.tobytes()
        if not fw:
            seq = revcomp(seq)
        q = (rng.integers(qmin, qmax + 1, size=rdlen) + 33).astype(np.uint8).tobytes()
        reads.append((f"r{i}:{c}:{p}:{int(fw)}", seq, q))
        i += 1
    return reads


def write_fastq(path: str, reads) -> None:
    with open(path, "wb") as f:
        for name, seq, q in reads:
            f.write(b"@" + name.encode() + b"\n" + seq + b"\n+\n" + q + b"\n")


def read_fastq(path: str) -> list[tuple[str, bytes, bytes]]:
    out = []
    with open(path, "rb") as f:
        while True:
            h = f.readline()
            if not h:
                break
            s = f.readline().strip()
            f.readline()
            q = f.readline().strip()
            out.append((h.strip()[1:].decode(), s, q))
    return out


def sim_reads_fixed(genome_codes: np.ndarray, chrom_starts: np.ndarray, n: int, rdlen: int,
                    seed: int, sub_rate: float = 0.01, indel_frac: float = 0.10,
                    rc_frac: float = 0.5, qmin: int = 2, qmax: int = 40, n_rate: float = 0.001):
    """Vectorised fixed-length read simulator over a concatenated genome (codes 0-4).

    Same error model as sim_reads; origins avoid N and chromosome boundaries.
    Returns (reads (n, rdlen) u8 codes as sequenced, quals (n, rdlen) u8 Phred+33,
    chrom (n,), off (n,) leftmost 0-based offset within the chromosome, fw (n,) bool)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    G = len(genome_codes)
    ends = np.append(chrom_starts[1:], G)
    over = int(n * 1.3) + 64
    out_pos = np.empty(0, dtype=np.int64)
    isn = (genome_codes > 3).astype(np.int32)
    csum = np.concatenate([[0], np.cumsum(isn)])
    while len(out_pos) < n:
        p = rng.integers(0, G - rdlen - 2, size=over)
        c = np.searchsorted(chrom_starts, p, side="right") - 1
        ok = (p + rdlen + 1 < ends[c]) & (csum[p + rdlen + 1] - csum[p] == 0)
        out_pos = np.concatenate([out_pos, p[ok]])
    p = out_pos[:n]
    chrom = np.searchsorted(chrom_starts, p, side="right") - 1
    j = np.arange(rdlen)[None, :]
    idx = np.broadcast_to(p[:, None] + j, (n, rdlen)).copy()
    indel = rng.random(n) < indel_frac
    k = rng.integers(10, rdlen - 10, size=n)[:, None]
    dele = indel & (rng.random(n) < 0.5)
    ins = indel & ~dele
    idx = np.where(dele[:, None] & (j >= k), idx + 1, idx)
    idx = np.where(ins[:, None] & (j > k), idx - 1, idx)
    reads = genome_codes[idx].astype(np.uint8)
    insmask = ins[:, None] & (j == k)
    reads = np.where(insmask, rng.integers(0, 4, size=(n, rdlen)).astype(np.uint8), reads)
    sub = rng.random((n, rdlen)) < sub_rate
    reads = np.where(sub, rng.integers(0, 4, size=(n, rdlen)).astype(np.uint8), reads)
    reads = np.where(rng.random((n, rdlen)) < n_rate, np.uint8(4), reads)
    fw = rng.random(n) >= rc_frac
    rc = np.where(reads < 4, 3 - reads, 4).astype(np.uint8)[:, ::-1]
    reads = np.where(fw[:, None], reads, rc)
    quals = (rng.integers(qmin, qmax + 1, size=(n, rdlen)) + 33).astype(np.uint8)
    return np.ascontiguousarray(reads), quals, chrom, p - chrom_starts[chrom], fw


def concat_genome(chroms):
    """[(name, ACGTN bytes)] -> (codes u8 concatenated, chrom start offsets)."""
    lut = np.full(256, 4, dtype=np.uint8)
    for i, ch in enumerate(b"ACGT"):
        lut[ch] = i
        lut[ch + 32] = i
    parts = [lut[np.frombuffer(s, dtype=np.uint8)] for _, s in chroms]
    starts = np.cumsum([0] + [len(x) for x in parts[:-1]]).astype(np.int64)
    return np.concatenate(parts), starts


# Config C2's reference: E. coli K-12 is not available offline, so a seeded
# synthetic genome of its length stands in (tests/golden/e2e_md5.json pins its FASTA md5).
ECOLI_LEN = 4_641_652


def ecoli_genome():
    return gen_genome(ECOLI_LEN, nchrom=1, seed=1)


def write_fastq_fixed(path: str, reads: np.ndarray, quals: np.ndarray, first_id: int = 0,
                      append: bool = False) -> None:
    """Fixed-length FASTQ from (n, R) code / Phred+33 arrays, vectorised: '@r<9 digits>'
    names (ids from first_id)."""
    n, R = reads.shape
    rec = np.empty((n, 11 + 1 + R + 3 + R + 1), dtype=np.uint8)
    rec[:, 0] = ord("@")
    rec[:, 1] = ord("r")
    ids = np.arange(first_id, first_id + n, dtype=np.int64)
    for k in range(9):
        rec[:, 10 - k] = ord("0") + (ids // (10 ** k)) % 10
    rec[:, 11] = ord("\n")
    rec[:, 12:12 + R] = ACGT[reads]
    rec[:, 12 + R] = ord("\n")
    rec[:, 13 + R] = ord("+")
    rec[:, 14 + R] = ord("\n")
    rec[:, 15 + R:15 + 2 * R] = quals
    rec[:, 15 + 2 * R] = ord("\n")
    with open(path, "ab" if append else "wb") as f:
        f.write(rec.tobytes())


def fixture_reads(chroms, path: str, n: int, rdlen: int, seed: int) -> None:
    """n simulated fixed-length reads (sim_reads_fixed, BASELINE.md error model) of the
    genome `chroms`, written to `path` (the e2e md5 fixtures of tests/golden/e2e_md5.json)."""
    codes, starts = concat_genome(chroms)
    reads, quals, _, _, _ = sim_reads_fixed(codes, starts, n, rdlen, seed=seed)
    write_fastq_fixed(path, reads, quals)



def sim_reads_fast(genome_codes: np.ndarray, chrom_starts: np.ndarray, n: int, rdlen: int, seed: int,
                   sub_rate: float = 0.01, indel_frac: float = 0.10, rc_frac: float = 0.5,
                   qmin: int = 2, qmax: int = 40, n_rate: float = 0.001):
    """sim_reads_fixed's error model (1 % substitutions, one indel in 10 % of
    reads, half reverse-complemented, Phred uniform qmin..qmax, rare Ns) with narrow
    integer draws and window gathers: ~10x faster, for bench-scale read sets (a different
    random stream than sim_reads_fixed, whose outputs the md5 fixtures pin)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    G = len(genome_codes)
    ends = np.append(chrom_starts[1:], G)
    isn = genome_codes > 3
    out_pos = np.empty(0, dtype=np.int64)
    W = rdlen + 2
    while len(out_pos) < n:
        p = rng.integers(0, G - W, size=int(n * 1.2) + 64)
        c = np.searchsorted(chrom_starts, p, side="right") - 1
        ok = p + W <= ends[c]
        p = p[ok]
        win = np.lib.stride_tricks.sliding_window_view(isn, W)[p]
        out_pos = np.concatenate([out_pos, p[~win.any(axis=1)]])
    p = out_pos[:n]
    win = np.lib.stride_tricks.sliding_window_view(genome_codes, W)[p]       # (n, W) u8
    j = np.arange(rdlen, dtype=np.int16)[None, :]
    k = rng.integers(10, rdlen - 10, size=(n, 1), dtype=np.int16)
    kind = rng.integers(0, 1 << 16, size=n, dtype=np.uint16)
    indel = kind < int(indel_frac * 65536)
    dele = indel & ((kind & 1) == 0)
    ins = indel & ~dele
    idx = j + (dele[:, None] & (j >= k)).astype(np.int16) - (ins[:, None] & (j > k)).astype(np.int16) + 1
    reads = np.take_along_axis(win, idx.astype(np.intp), axis=1)
    rnd = rng.integers(0, 1 << 16, size=(n, rdlen), dtype=np.uint16)
    codes = rng.integers(0, 256, size=(n, rdlen), dtype=np.uint8) & 3
    reads = np.where(ins[:, None] & (j == k), codes, reads)
    reads = np.where(rnd < int(sub_rate * 65536), codes, reads)
    reads = np.where(rnd >= 65536 - int(n_rate * 65536), np.uint8(4), reads)
    fw = rng.random(n) >= rc_frac
    rc = np.where(reads < 4, 3 - reads, 4).astype(np.uint8)[:, ::-1]
    reads = np.where(fw[:, None], reads, rc)
    quals = (rng.integers(qmin, qmax + 1, size=(n, rdlen), dtype=np.uint8) + 33).astype(np.uint8)
    return np.ascontiguousarray(reads), quals
