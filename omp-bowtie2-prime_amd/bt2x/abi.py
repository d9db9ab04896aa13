"""numpy / ctypes mirror of include/bt2x.h (the C-ABI boundary).

The record layouts below are the C structs of bt2x.h with natural alignment; tests
assert their sizes against the library (bt2x_abi_sizes) so the two cannot drift.
"""
from __future__ import annotations

import ctypes
import numpy as np

ABI_VERSION = 4             # BT2X_ABI_VERSION of the bt2x.h these mirrors follow

SEED_IN = np.dtype([("read_off", "<u8"), ("seed_off", "u1"), ("seed_len", "u1"),
                    ("pad", "u1", 6)], align=True)
SEED_OUT = np.dtype([("topf", "<u8"), ("botf", "<u8"), ("nlex", "u1"),
                     ("need_reporting", "u1"), ("pad", "u1", 6)], align=True)
DP_IN = np.dtype([("read_off", "<u8"), ("qual_off", "<u8"), ("ref_off", "<u8"),
                  ("refl", "<i8"), ("rdlen", "<u2"), ("ncol", "<u2"), ("minsc", "<i2"),
                  ("nceil", "<i2"), ("triml", "<u2"), ("corel", "<u2"), ("corer", "<u2"),
                  ("fw", "u1"), ("flags", "u1")], align=True)
DP_I16 = 1                  # bt2x_dp_in.flags: the reference's signed 16-bit DP (--no-sse8)
DP_REF_TEXT = 2             # bt2x_dp_in.flags: window cut from the index (ref_off = text id)
DPL_I16, DPL_EXACT_BEST, DPL_REF_TEXT = 1, 2, 4
CAP_REF_TEXT = 1            # bt2x_capabilities
OPT_EXACT_BEST = 1
DP_OUT = np.dtype([("status", "<i4"), ("best", "<i4"), ("ncand", "<u2"), ("nrec", "<u2"),
                   ("rec_off", "<u4")], align=True)
ALN_REC = np.dtype([("ntries", "<u2"), ("ok", "u1"), ("pad0", "u1"), ("score", "<i2"),
                    ("ns", "<u2"), ("gaps", "<u2"), ("nedit", "<u2"),
                    ("bases_aligned", "<u2"), ("refns", "<u2"), ("refoff", "<i8"),
                    ("edit_off", "<u4"), ("nbuf", "<u4")], align=True)
RESOLVE_IN = np.dtype([("row", "<u8"), ("qlen", "<u4"), ("pad", "<u4")], align=True)
RESOLVE_OUT = np.dtype([("joff", "<u8"), ("toff", "<u8"), ("tlen", "<u8"), ("tidx", "<u4"),
                        ("straddled", "<u4")], align=True)
NO_TIDX = 0xFFFFFFFF
ELT = np.dtype([("v", "<u8")])   # bt2x_elt: toff bits 0-38, straddled bit 39, tidx bits 40-63
STORE_IN = np.dtype([("off", "<u8"), ("slot", "<u4"), ("len", "<u2"), ("pad", "<u2")], align=True)   # bt2x_store_in
STORE_SLOT_BYTES = 1024
SAM_MAX_MM = 16
SAM_REQ = np.dtype([("slot", "<u4"), ("rdlen", "<u2"), ("fw", "u1"), ("nmm", "u1"), ("as_", "<i4"), ("xs", "<i4"),
                    ("xn", "<u4"), ("has_xs", "<u4"), ("text_off", "<u8"), ("mm_pos", "<u2", (SAM_MAX_MM,)),
                    ("mm_chr", "u1", (SAM_MAX_MM,))], align=True)   # bt2x_sam_req


def sam_tail_max(rdlen, nmm):
    """BT2X_SAM_TAIL_MAX"""
    return 2 * rdlen + 200 + 4 * nmm
ROUND_IN = np.dtype([("read_off", "<u8"), ("seed0", "<u8"), ("rnd_last", "<u4"), ("rnd_lastoff", "<i4"),
                     ("exr0", "<u4"), ("nexr", "<u2"), ("nseeds", "<u2"), ("num_offs", "<u2"),
                     ("rdlen", "<u2"), ("interval", "<u2"), ("offset", "<u2"), ("seedlen", "<u2"),
                     ("seedflags", "<u2"), ("pad", "<u2", 2)], align=True)
EXRANGE = np.dtype([("sz", "<u8"), ("off", "<u4"), ("len", "<u2"), ("fw", "u1"), ("pad", "u1")], align=True)
SAT = np.dtype([("rdoff", "<u2"), ("rand_n", "u1"), ("fwlen", "u1")], align=True)   # fwlen: fw << 7 | seedlen
ROUND_OUT = np.dtype([("rnd_last", "<u4"), ("rnd_lastoff", "<i4"), ("num_elts", "<u8"), ("nonz", "<u4"),
                      ("status", "<u4"), ("sat0", "<u4"), ("nsat", "<u4"), ("elt0", "<u4"), ("nelt", "<u4"),
                      ("exr0", "<u4"), ("nexr", "<u4")], align=True)
ROUND_OK, ROUND_NO_HITS, ROUND_REDO = 0, 1, 2

MAX_ROWS = 160
MAX_COLS = 200
E_OK, E_ARG, E_IO, E_NODEVICE, E_OVERFLOW, E_NOMEM = 0, -1, -2, -3, -4, -5
K_SEED, K_DP, K_RESOLVE, K_ROUND = 0, 1, 2, 3

EDIT_READ_GAP, EDIT_REF_GAP, EDIT_MM = 1, 2, 3


def edit_fields(e: int) -> tuple[int, int, str, str]:
    """Unpack a bt2x packed edit -> (pos, type, chr, qchr)."""
    e = int(e)
    return e & 0x3FF, (e >> 12) & 7, chr((e >> 16) & 0xFF), chr((e >> 24) & 0xFF)


def cand_fields(c: int, i16: bool = False) -> tuple[int | None, int, int]:
    """Unpack a debug candidate -> (row, col, DpBtCandidate::score).  i16 entries
    (BT2X_CAND_PACK16) carry no row (always rdlen - 1) and an int16 score."""
    c = int(c)
    if i16:
        sc = c & 0xFFFF
        return None, c >> 16, sc - 0x10000 if sc >= 0x8000 else sc
    return (c >> 8) & 0xFF, c >> 16, c & 0xFF


class IndexDesc(ctypes.Structure):
    _fields_ = [("len", ctypes.c_uint64), ("zoff", ctypes.c_uint64),
                ("fchr", ctypes.c_uint64 * 5), ("ftab_chars", ctypes.c_int32),
                ("off_rate", ctypes.c_int32), ("line_rate", ctypes.c_int32),
                ("flags", ctypes.c_int32),
                ("ebwt", ctypes.c_void_p), ("ebwt_bytes", ctypes.c_uint64),
                ("ftab", ctypes.c_void_p), ("ftab_len", ctypes.c_uint64),
                ("eftab", ctypes.c_void_p), ("eftab_len", ctypes.c_uint64),
                ("offs", ctypes.c_void_p), ("offs_len", ctypes.c_uint64),
                ("plen", ctypes.c_void_p), ("npat", ctypes.c_uint64),
                ("rstarts", ctypes.c_void_p), ("nfrag", ctypes.c_uint64),
                ("text2", ctypes.c_void_p), ("text2_bytes", ctypes.c_uint64),
                ("owner", ctypes.c_void_p)]

    def array(self, name: str, dtype, count_field: str) -> np.ndarray:
        n = int(getattr(self, count_field))
        p = getattr(self, name)
        if not p or n == 0:
            return np.zeros(0, dtype=dtype)
        buf = (ctypes.c_uint8 * (n * np.dtype(dtype).itemsize)).from_address(p)
        return np.frombuffer(buf, dtype=dtype, count=n)


class Scoring(ctypes.Structure):
    _fields_ = [("mm_max", ctypes.c_int32), ("mm_min", ctypes.c_int32),
                ("n_pen", ctypes.c_int32), ("rdg_const", ctypes.c_int32),
                ("rdg_linear", ctypes.c_int32), ("rfg_const", ctypes.c_int32),
                ("rfg_linear", ctypes.c_int32), ("gapbar", ctypes.c_int32),
                ("mmpens", ctypes.c_int32 * 256), ("npens", ctypes.c_int32 * 256)]


class Counters(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in
                ("n_bilf", "n_lf1", "n_ftab", "dp_cells", "dp_cols", "bt_cells",
                 "n_problems", "alg_bytes", "dp_cells_computed")]

    def as_dict(self) -> dict:
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class DpDebug(ctypes.Structure):
    _fields_ = [("digests", ctypes.c_void_p), ("cands", ctypes.c_void_p)]


def ptr(a: np.ndarray | None) -> ctypes.c_void_p:
    if a is None:
        return ctypes.c_void_p(0)
    return ctypes.c_void_p(a.ctypes.data)
