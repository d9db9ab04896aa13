"""Readers for the golden vectors in tests/golden/ (written by tools/make_golden.py from
oracle/refharness.cpp, i.e. by the reference's own SeedAligner / SwAligner code) and
builders of the bt2x C-ABI input batches that reproduce each golden case.
"""
from __future__ import annotations

import gzip
import lzma
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLDEN = os.path.join(HERE, "golden")
sys.path.insert(0, os.path.join(ROOT, "omp-bowtie2-prime_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from bt2x import abi  # noqa: E402

_CODE = np.full(256, 4, dtype=np.uint8)
for _i, _c in enumerate(b"ACGT"):
    _CODE[_c] = _i
    _CODE[_c + 32] = _i


def codes(seq: bytes) -> np.ndarray:
    return _CODE[np.frombuffer(seq, dtype=np.uint8)]


def rc_codes(c: np.ndarray) -> np.ndarray:
    out = np.where(c < 4, 3 - c, 4).astype(np.uint8)
    return out[::-1].copy()


def open_text(path: str):
    if path.endswith(".gz"):
        return gzip.open(path, "rt")
    if path.endswith(".xz"):
        return lzma.open(path, "rt")
    return open(path, "rt")


def read_fastq(path: str):
    out = []
    with open_text(path) as f:
        while True:
            h = f.readline()
            if not h:
                break
            s = f.readline().strip()
            f.readline()
            q = f.readline().strip()
            out.append((h.strip()[1:], s.encode(), q.encode()))
    return out


def materialize_index(name: str, dest: str) -> str:
    """Decompress tests/golden/<name>.{1,2,3,4}.bt2l.xz into dest; return basename."""
    os.makedirs(dest, exist_ok=True)
    base = os.path.join(dest, name)
    for k in ("1", "2", "3", "4"):
        src = os.path.join(GOLDEN, f"{name}.{k}.bt2l.xz")
        dst = f"{base}.{k}.bt2l"
        if os.path.exists(src) and not os.path.exists(dst):
            with lzma.open(src, "rb") as fi, open(dst, "wb") as fo:
                fo.write(fi.read())
    return base


class SeedCase:
    """Seeds golden: reads buffer + bt2x_seed_in batch + expected bt2x_seed_out."""

    def __init__(self, fastq: str, golden: str):
        reads = read_fastq(fastq)
        bufs, offs = [], []
        pos = 0
        for _, s, _ in reads:
            c = codes(s)
            offs.append((pos, pos + len(c)))
            bufs.append(c)
            bufs.append(rc_codes(c))
            pos += 2 * len(c)
        self.reads = np.concatenate(bufs) if bufs else np.zeros(0, np.uint8)
        rows = []
        with open_text(golden) as f:
            for line in f:
                if not line.startswith("S "):
                    continue
                t = line.split()
                rows.append([int(x) for x in t[1:11]])
        a = np.array(rows, dtype=np.int64).reshape(-1, 10)
        self.n = len(a)
        self.inp = np.zeros(self.n, dtype=abi.SEED_IN)
        ridx, fw = a[:, 0], a[:, 2]
        base = np.array(offs, dtype=np.int64).reshape(-1, 2)
        self.inp["read_off"] = np.where(fw == 1, base[ridx, 0], base[ridx, 1])
        self.inp["seed_off"] = a[:, 4]
        self.inp["seed_len"] = a[:, 5]
        self.exp_topf = a[:, 6].astype(np.uint64)
        self.exp_botf = a[:, 7].astype(np.uint64)
        self.exp_rep = a[:, 8].astype(np.uint8)
        self.exp_nlex = a[:, 9].astype(np.uint8)


class DpCase:
    """DP golden: buffers + bt2x_dp_in batch + expected align()/nextAlignment() results."""

    def __init__(self, golden: str):
        probs = []
        cur = None
        with open_text(golden) as f:
            for line in f:
                t = line.split()
                if not t:
                    continue
                if t[0] == "P":
                    cur = {"fw": int(t[3]), "seq": t[4].encode(), "qual": t[5].encode(),
                           "win": t[6].encode(), "refl": int(t[7]), "refr": int(t[8]),
                           "triml": int(t[9]), "corel": int(t[10]), "corer": int(t[11]),
                           "minsc": int(t[12]), "nceil": int(t[13]), "rseed": int(t[14]),
                           "refoff": int(t[15]), "tidx": int(t[16]), "tlen": int(t[17]),
                           "i16": int(t[18]) if len(t) > 18 else 0,      # refharness-i16: enable8_ off
                           "cands": [], "calls": []}
                    probs.append(cur)
                elif t[0] == "A":
                    cur["ok"] = int(t[1])
                    cur["best"] = int(t[2])
                    cur["ncand"] = int(t[3])
                    cur["digest"] = [int(x, 16) for x in t[4:7]]
                elif t[0] == "C":
                    cur["cands"] = [tuple(int(v) for v in x.split(",")) for x in t[1:]]
                elif t[0] == "N":
                    if t[1] == "0":
                        cur["calls"].append({"ok": 0, "rnd": int(t[2])})
                    else:
                        edits = []
                        for x in t[11:]:
                            p, ty, ch, qc = x.split(",")
                            edits.append((int(p), int(ty), ch, qc))
                        cur["calls"].append({"ok": 1, "rnd": int(t[2]), "score": int(t[3]),
                                             "ns": int(t[4]), "gaps": int(t[5]),
                                             "nedit": int(t[6]), "bases": int(t[7]),
                                             "refoff": int(t[8]), "refns": int(t[9]),
                                             "edits": edits})
        self.probs = probs
        self.n = len(probs)
        rd, qu, rf = [], [], []
        self.inp = np.zeros(self.n, dtype=abi.DP_IN)
        pr = pq = pf = 0
        for i, p in enumerate(probs):
            c = codes(p["seq"])
            q = np.frombuffer(p["qual"], dtype=np.uint8)
            if not p["fw"]:
                c = rc_codes(c)
                q = q[::-1].copy()
            w = codes(p["win"])
            rd.append(c); qu.append(q); rf.append(w)
            x = self.inp[i]
            x["read_off"], x["qual_off"], x["ref_off"] = pr, pq, pf
            x["refl"] = p["refl"]
            x["rdlen"], x["ncol"] = len(c), len(w)
            x["minsc"], x["nceil"] = p["minsc"], p["nceil"]
            x["triml"], x["corel"], x["corer"] = p["triml"], p["corel"], p["corer"]
            x["fw"] = p["fw"]
            x["flags"] = abi.DP_I16 if p["i16"] else 0
            pr += len(c); pq += len(q); pf += len(w)
        self.reads = np.concatenate(rd) if rd else np.zeros(1, np.uint8)
        self.quals = np.concatenate(qu) if qu else np.zeros(1, np.uint8)
        self.refs = np.concatenate(rf) if rf else np.zeros(1, np.uint8)


def replay_rng(seed: int, ntries_per_call, i16: bool = False):
    """Reproduce RandomSource after each nextAlignment call: per attempted candidate
    reseed = nextU32() + 1, then init(reseed + 1) on the u8 path (aligner_sw.cpp:324-336)
    or init(reseed) on the i16 path (:338-348)."""
    last = seed & 0xFFFFFFFF
    out = []
    for nt in ntries_per_call:
        for _ in range(nt):
            last = (1664525 * last + 1013904223) & 0xFFFFFFFF
            ret = last >> 16
            last = (1664525 * last + 1013904223) & 0xFFFFFFFF
            ret ^= last
            reseed = (ret + 1) & 0xFFFFFFFF
            last = reseed if i16 else (reseed + 1) & 0xFFFFFFFF
        out.append(last)
    return out


def compare_dp(case: DpCase, out, recs, edits, digests=None, cands=None, limit=20):
    """Return a list of mismatch descriptions (empty = bit-exact)."""
    bad = []
    for i, p in enumerate(case.probs):
        o = out[i]
        if int(o["status"]) != p["ok"] or int(o["best"]) != p["best"] or int(o["ncand"]) != p["ncand"]:
            if not (p["ok"] == 0 and p["best"] < -(1 << 40) and int(o["best"]) == -(1 << 31)):
                bad.append(f"prob {i}: align status/best/ncand {int(o['status'])}/{int(o['best'])}/"
                           f"{int(o['ncand'])} != {p['ok']}/{p['best']}/{p['ncand']}")
        if digests is not None and list(int(v) for v in digests[i]) != p["digest"]:
            bad.append(f"prob {i}: E/F/H digest mismatch")
        if cands is not None:
            got = [abi.cand_fields(c, p["i16"]) for c in cands[i][: int(o["ncand"])]]
            want = [tuple(c) for c in p["cands"]]
            if p["i16"]:
                rows = {c[0] for c in want}
                want = [(None, c[1], c[2]) for c in want]
                if rows and rows != {len(p["seq"]) - 1}:
                    bad.append(f"prob {i}: i16 candidate outside the last row")
            if got != want:
                bad.append(f"prob {i}: candidate list mismatch")
        calls = p["calls"]
        nrec = int(o["nrec"])
        if nrec != len(calls):
            bad.append(f"prob {i}: {nrec} nextAlignment calls != {len(calls)}")
        else:
            r = recs[int(o["rec_off"]): int(o["rec_off"]) + nrec]
            rnd = replay_rng(p["rseed"], [int(x["ntries"]) for x in r], p["i16"])
            for k, (rec, exp) in enumerate(zip(r, calls)):
                if rnd[k] != exp["rnd"] or int(rec["ok"]) != exp["ok"]:
                    bad.append(f"prob {i} call {k}: rng/ok mismatch")
                    continue
                if not exp["ok"]:
                    continue
                got = (int(rec["score"]), int(rec["ns"]), int(rec["gaps"]), int(rec["nedit"]),
                       int(rec["bases_aligned"]), int(rec["refoff"]), int(rec["refns"]))
                want = (exp["score"], exp["ns"], exp["gaps"], exp["nedit"], exp["bases"],
                        exp["refoff"], exp["refns"])
                if got != want:
                    bad.append(f"prob {i} call {k}: {got} != {want}")
                    continue
                ge = [abi.edit_fields(e) for e in
                      edits[int(rec["edit_off"]): int(rec["edit_off"]) + int(rec["nedit"])]]
                if ge != exp["edits"]:
                    bad.append(f"prob {i} call {k}: edits {ge} != {exp['edits']}")
        if len(bad) >= limit:
            break
    return bad


def dp_header(golden: str) -> dict:
    with open_text(golden) as f:
        h = f.readline().split()
    return dict(x.split("=", 1) for x in h if "=" in x)


def dp_header_sse8(golden: str) -> int:
    """--sse8 / --no-sse8 of a DP golden (refharness-i16 records it; older sets: 1)."""
    return int(dp_header(golden).get("sse8", 1))


def dp_header_scoring(golden: str) -> dict:
    """Scoring parameters recorded in a DP golden header line by refharness."""
    kv = dp_header(golden)
    mx, mn = (int(v) for v in kv["mmp"].split(","))
    rdc, rdl = (int(v) for v in kv["rdg"].split(","))
    rfc, rfl = (int(v) for v in kv["rfg"].split(","))
    return {"mm_max": mx, "mm_min": mn, "n_pen": int(kv["np"]), "rdg_const": rdc,
            "rdg_linear": rdl, "rfg_const": rfc, "rfg_linear": rfl, "gapbar": int(kv["gapbar"])}


class ResolveCase:
    """tests/golden/resolve_*.txt.xz (refharness resolve): seed-range elements through
    GroupWalk2S::advanceElement ('W', ranges of <= 6 elements) or Ebwt::getOffset ('V',
    larger ranges), and joinedToTextOff fragment-boundary probes ('J'); every record
    carries joinedToTextOff's (tidx, toff, tlen, straddled) for rejectStraddle = false
    and true (tidx -1 = OFF_MASK)."""

    def __init__(self, path: str):
        walk, probe = [], []
        self.kinds = []
        with open_text(path) as f:
            for line in f:
                t = line.split()
                if not t or t[0] in ("#", "G"):
                    continue
                if t[0] in ("W", "V"):
                    walk.append([int(x) for x in t[2:]])           # row joff qlen + 8
                    self.kinds.append(t[0])
                elif t[0] == "J":
                    probe.append([int(x) for x in t[1:]])          # off qlen + 8
        w = np.array(walk, dtype=np.int64).reshape(-1, 11)
        p = np.array(probe, dtype=np.int64).reshape(-1, 10)
        self.rows, self.joff, self.qlen = w[:, 0].astype(np.uint64), w[:, 1].astype(np.uint64), w[:, 2]
        self.exp = [self._res(w[:, 3:7]), self._res(w[:, 7:11])]
        self.j_off, self.j_qlen = p[:, 0].astype(np.uint64), p[:, 1]
        self.j_exp = [self._res(p[:, 2:6]), self._res(p[:, 6:10])]
        self.n = len(w)

    @staticmethod
    def _res(a):
        tidx = np.where(a[:, 0] < 0, abi.NO_TIDX, a[:, 0]).astype(np.uint32)
        return {"tidx": tidx, "toff": a[:, 1].astype(np.uint64), "tlen": a[:, 2].astype(np.uint64),
                "straddled": a[:, 3].astype(np.uint32)}


def compare_resolve(out, exp, joff=None):
    """Mismatch count of RESOLVE_OUT records against a ResolveCase expectation dict."""
    bad = 0
    for k, v in exp.items():
        bad += int((out[k] != v).sum())
    if joff is not None:
        bad += int((out["joff"] != joff).sum())
    return bad
