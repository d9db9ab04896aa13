"""ctypes binding of oracle/liboracle.so — the CPU checker (tests / smoke / bench
cpu_baseline only; the product never loads it)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from golden_io import ROOT, abi

ORACLE_DIR = os.path.join(ROOT, "oracle")
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-C", ORACLE_DIR, "liboracle.so"], check=True,
                           stdout=subprocess.DEVNULL)
        L = ctypes.CDLL(path)
        vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
        L.bt2o_index_load.argtypes = [ctypes.c_char_p, i32, ctypes.POINTER(abi.IndexDesc)]
        L.bt2o_index_free.argtypes = [ctypes.POINTER(abi.IndexDesc)]
        L.bt2o_scoring_default.argtypes = [ctypes.POINTER(abi.Scoring)]
        L.bt2o_seed_search.argtypes = [ctypes.POINTER(abi.IndexDesc), vp, vp, u32, i32, vp,
                                       ctypes.POINTER(abi.Counters)]
        L.bt2o_dp_align.argtypes = [ctypes.POINTER(abi.Scoring), vp, vp, vp, vp, u32, vp,
                                    vp, u32, ctypes.POINTER(ctypes.c_uint32),
                                    vp, u32, ctypes.POINTER(ctypes.c_uint32),
                                    ctypes.POINTER(abi.DpDebug), ctypes.POINTER(abi.Counters)]
        L.bt2o_resolve.argtypes = [ctypes.POINTER(abi.IndexDesc), vp, u32, i32, vp,
                                   ctypes.POINTER(abi.Counters)]
        L.bt2o_count_side.restype = ctypes.c_uint64
        L.bt2o_count_side.argtypes = [ctypes.POINTER(abi.IndexDesc), ctypes.c_uint64, i32]
        _LIB = L
    return _LIB


class OracleIndex:
    def __init__(self, base: str, load_offs: bool = False):
        self.desc = abi.IndexDesc()
        rc = lib().bt2o_index_load(base.encode(), int(load_offs), ctypes.byref(self.desc))
        if rc != 0:
            raise IOError(f"oracle index load failed ({rc}) for {base}")

    def __del__(self):
        try:
            lib().bt2o_index_free(ctypes.byref(self.desc))
        except Exception:
            pass


def default_scoring() -> abi.Scoring:
    sc = abi.Scoring()
    lib().bt2o_scoring_default(ctypes.byref(sc))
    return sc


def seed_search(idx: OracleIndex, reads: np.ndarray, inp: np.ndarray, do_extend=True):
    out = np.zeros(len(inp), dtype=abi.SEED_OUT)
    ctr = abi.Counters()
    rc = lib().bt2o_seed_search(ctypes.byref(idx.desc), abi.ptr(reads), abi.ptr(inp), len(inp),
                                int(do_extend), abi.ptr(out), ctypes.byref(ctr))
    assert rc == 0, rc
    return out, ctr.as_dict()


def resolve(idx: OracleIndex, rows, qlen, reject_straddle=False):
    rows = np.asarray(rows, dtype=np.uint64)
    inp = np.zeros(len(rows), dtype=abi.RESOLVE_IN)
    inp["row"] = rows
    inp["qlen"] = qlen
    out = np.zeros(len(rows), dtype=abi.RESOLVE_OUT)
    ctr = abi.Counters()
    rc = lib().bt2o_resolve(ctypes.byref(idx.desc), abi.ptr(inp), len(inp), int(reject_straddle),
                            abi.ptr(out), ctypes.byref(ctr))
    assert rc == 0, rc
    return out, ctr.as_dict()


def dp_align(sc, reads, quals, refs, inp, debug=True, rec_cap=None, edit_cap=None):
    n = len(inp)
    rec_cap = rec_cap or max(16, 4 * n)
    edit_cap = edit_cap or max(256, 64 * n)
    out = np.zeros(n, dtype=abi.DP_OUT)
    recs = np.zeros(rec_cap, dtype=abi.ALN_REC)
    edits = np.zeros(edit_cap, dtype=np.uint32)
    nrec, nedit = ctypes.c_uint32(0), ctypes.c_uint32(0)
    dig = np.zeros((n, 3), dtype=np.uint64) if debug else None
    cands = np.zeros((n, abi.MAX_COLS), dtype=np.uint32) if debug else None
    dbg = abi.DpDebug(abi.ptr(dig).value, abi.ptr(cands).value) if debug else None
    ctr = abi.Counters()
    rc = lib().bt2o_dp_align(ctypes.byref(sc), abi.ptr(reads), abi.ptr(quals), abi.ptr(refs),
                             abi.ptr(inp), n, abi.ptr(out), abi.ptr(recs), rec_cap,
                             ctypes.byref(nrec), abi.ptr(edits), edit_cap, ctypes.byref(nedit),
                             ctypes.byref(dbg) if dbg is not None else None, ctypes.byref(ctr))
    if rc == abi.E_OVERFLOW:
        return dp_align(sc, reads, quals, refs, inp, debug, nrec.value + 1, nedit.value + 1)
    assert rc == 0, rc
    return out, recs[: nrec.value], edits[: nedit.value], dig, cands, ctr.as_dict()
