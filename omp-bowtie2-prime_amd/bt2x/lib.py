"""ctypes binding of libbt2x.so (the product library: gfx950 kernels + C-ABI).

There is deliberately no CPU fallback: if the shared library is missing, or no HIP
device is present, every entry point raises.  The CPU restatement in oracle/ is a test
checker and is never imported from here.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BT2X_LIB") or os.path.join(HERE, "libbt2x.so")   # BT2X_LIB: a development build
_LIB = None

FUNCS = {
    "bt2x_index_load": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(abi.IndexDesc)]),
    "bt2x_index_free": (None, [ctypes.POINTER(abi.IndexDesc)]),
    "bt2x_scoring_default": (None, [ctypes.POINTER(abi.Scoring)]),
    "bt2x_scoring_init": (None, [ctypes.POINTER(abi.Scoring)]),
    "bt2x_open": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(abi.IndexDesc),
                                 ctypes.POINTER(abi.Scoring), ctypes.POINTER(ctypes.c_void_p)]),
    "bt2x_open_shared": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "bt2x_device_numa_node": (ctypes.c_int, [ctypes.c_int]),
    "bt2x_close": (None, [ctypes.c_void_p]),
    "bt2x_last_kernel_ms": (ctypes.c_double, [ctypes.c_void_p, ctypes.c_int]),
    "bt2x_last_counters": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(abi.Counters)]),
    "bt2x_seed_search": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                        ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]),
    "bt2x_seed_search_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_void_p]),
    "bt2x_dp_align": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                     ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                     ctypes.POINTER(ctypes.c_uint32), ctypes.c_void_p,
                                     ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                     ctypes.POINTER(abi.DpDebug)]),
    "bt2x_dp_align_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                         ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                         ctypes.POINTER(abi.DpDebug), ctypes.c_uint32, ctypes.c_void_p]),
    "bt2x_set_option": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64]),
    "bt2x_capabilities": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)]),
    "bt2x_resolve": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                                    ctypes.c_void_p]),
    "bt2x_resolve_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p]),
    "bt2x_seed_round": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                       ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                       ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                       ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]),
    "bt2x_seed_round_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                           ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                           ctypes.c_void_p]),
    "bt2x_store_reads": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                        ctypes.c_uint32]),
    "bt2x_sam_tails": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64,
                                      ctypes.c_void_p]),
    "bt2x_sam_tails_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p]),
    "bt2x_version": (ctypes.c_char_p, []),
    "bt2x_abi_version": (ctypes.c_int, []),
    "bt2x_host_alloc": (ctypes.c_void_p, [ctypes.c_size_t]),
    "bt2x_last_round_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)]),
    "bt2x_last_round_stats_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32]),
    "bt2x_host_free": (None, [ctypes.c_void_p]),
    "bt2x_suffix_array": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]),
    "bt2x_build_index": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]),
    "bt2x_build_index_sa": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                           ctypes.c_void_p]),
    "bt2x_abi_sizes": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]),
}


class Bt2xError(RuntimeError):
    """A bt2x_* call returned a negative BT2X_E_* code (kept in .code)."""

    def __init__(self, msg: str, code: int = 0):
        super().__init__(msg)
        self.code = code


def load():
    """Load libbt2x.so (built in-tree by __graft_entry__.build()); raise if absent."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise Bt2xError(f"{LIB_PATH} is missing: build it with "
                            "`make -C omp-bowtie2-prime_amd/csrc` (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in FUNCS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        v = L.bt2x_abi_version()
        if v != abi.ABI_VERSION:      # a stale binding would misread the record arenas
            raise Bt2xError(f"{LIB_PATH} has ABI version {v}, this binding follows {abi.ABI_VERSION}")
        _LIB = L
    return _LIB


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise Bt2xError(f"{what} failed with bt2x error {rc}", rc)


def default_scoring(**overrides) -> abi.Scoring:
    sc = abi.Scoring()
    L = load()
    L.bt2x_scoring_default(ctypes.byref(sc))
    if overrides:
        for k, v in overrides.items():
            setattr(sc, k, int(v))
        L.bt2x_scoring_init(ctypes.byref(sc))
    return sc


class Index:
    """Host image of a forward .bt2l index (Ebwt::readIntoMemory)."""

    def __init__(self, basename: str, load_offs: bool = False):
        self.desc = abi.IndexDesc()
        check(load().bt2x_index_load(basename.encode(), int(load_offs), ctypes.byref(self.desc)),
              f"bt2x_index_load({basename})")
        self.basename = basename

    def close(self):
        if self.desc.owner:
            load().bt2x_index_free(ctypes.byref(self.desc))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """One GPU context (bt2x_open): uploaded index + scoring + kernel launch state."""

    def __init__(self, index: Index, device: int = 0, scoring: abi.Scoring | None = None):
        self.index = index
        self.scoring = scoring if scoring is not None else default_scoring()
        h = ctypes.c_void_p()
        check(load().bt2x_open(device, ctypes.byref(index.desc), ctypes.byref(self.scoring),
                               ctypes.byref(h)), "bt2x_open")
        self.h = h

    def close(self):
        if self.h:
            load().bt2x_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -------------------------------------------------------------- seeds
    def seed_search(self, reads: np.ndarray, inp: np.ndarray, do_extend: bool = True) -> np.ndarray:
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        inp = np.ascontiguousarray(inp, dtype=abi.SEED_IN)
        out = np.zeros(len(inp), dtype=abi.SEED_OUT)
        check(load().bt2x_seed_search(self.h, abi.ptr(reads), reads.nbytes, abi.ptr(inp), len(inp),
                                      int(do_extend), abi.ptr(out)), "bt2x_seed_search")
        return out

    def seed_search_dev(self, d_reads: int, d_in: int, n: int, d_out: int, do_extend=True, stream=0):
        check(load().bt2x_seed_search_dev(self.h, d_reads, d_in, n, int(do_extend), d_out, stream),
              "bt2x_seed_search_dev")

    # ----------------------------------------------------------------- DP
    def store_reads(self, packed, inp):
        """bt2x_store_reads: read i's patFw codes then its qualities at packed[inp[i].off]
        into store slot inp[i].slot."""
        packed = np.ascontiguousarray(packed, dtype=np.uint8)
        inp = np.ascontiguousarray(inp, dtype=abi.STORE_IN)
        check(load().bt2x_store_reads(self.h, abi.ptr(packed), packed.nbytes, abi.ptr(inp), len(inp)),
              "bt2x_store_reads")

    def sam_tails(self, req):
        """bt2x_sam_tails: the record tails (bytes) of requests req (abi.SAM_REQ; text_off is
        filled here), from the read store."""
        req = np.array(req, dtype=abi.SAM_REQ)
        bound = np.array([abi.sam_tail_max(int(r["rdlen"]), int(r["nmm"])) for r in req], dtype=np.uint64)
        req["text_off"] = np.concatenate([[0], np.cumsum(bound)[:-1]]).astype(np.uint64) if len(req) else bound
        text = np.zeros(int(bound.sum()) if len(req) else 1, dtype=np.uint8)
        lens = np.zeros(max(1, len(req)), dtype=np.uint16)
        check(load().bt2x_sam_tails(self.h, abi.ptr(req), len(req), abi.ptr(text), text.nbytes, abi.ptr(lens)),
              "bt2x_sam_tails")
        return [text[int(r["text_off"]): int(r["text_off"]) + int(lens[i])].tobytes() for i, r in enumerate(req)]

    def dp_align(self, reads, quals, refs, inp, debug=False, rec_cap=None, edit_cap=None):
        """reads = quals = None: read_off / qual_off index the read store."""
        store = reads is None and quals is None
        reads = np.zeros(1, np.uint8) if store else np.ascontiguousarray(reads, dtype=np.uint8)
        quals = np.zeros(1, np.uint8) if store else np.ascontiguousarray(quals, dtype=np.uint8)
        refs = np.ascontiguousarray(refs, dtype=np.uint8)
        inp = np.ascontiguousarray(inp, dtype=abi.DP_IN)
        n = len(inp)
        rec_cap = rec_cap or max(64, 4 * n)
        edit_cap = edit_cap or max(1024, 32 * n)
        out = np.zeros(n, dtype=abi.DP_OUT)
        recs = np.zeros(rec_cap, dtype=abi.ALN_REC)
        edits = np.zeros(edit_cap, dtype=np.uint32)
        nrec, nedit = ctypes.c_uint32(0), ctypes.c_uint32(0)
        dig = np.zeros((n, 3), dtype=np.uint64) if debug else None
        cands = np.zeros((n, abi.MAX_COLS), dtype=np.uint32) if debug else None
        dbg = abi.DpDebug(abi.ptr(dig).value, abi.ptr(cands).value) if debug else None
        rc = load().bt2x_dp_align(self.h, None if store else abi.ptr(reads), reads.nbytes,
                                  None if store else abi.ptr(quals), quals.nbytes,
                                  abi.ptr(refs), refs.nbytes, abi.ptr(inp), n, abi.ptr(out),
                                  abi.ptr(recs), rec_cap, ctypes.byref(nrec), abi.ptr(edits),
                                  edit_cap, ctypes.byref(nedit),
                                  ctypes.byref(dbg) if dbg is not None else None)
        if rc == abi.E_OVERFLOW:
            return self.dp_align(None if store else reads, None if store else quals, refs, inp, debug,
                                 nrec.value + 64, nedit.value + 1024)
        check(rc, "bt2x_dp_align")
        return out, recs[: nrec.value], edits[: nedit.value], dig, cands

    def dp_align_dev(self, d_reads, d_quals, d_refs, d_in, n, d_out, d_recs, rec_cap, d_edits,
                     edit_cap, d_counters, stream=0, launch_flags=0):
        """bt2x_dp_align_dev; launch_flags: abi.DPL_I16 (some problem is BT2X_DP_I16),
        abi.DPL_EXACT_BEST (exact best of failed problems), abi.DPL_REF_TEXT (some problem
        is BT2X_DP_REF_TEXT).  d_counters: 4 x u32."""
        check(load().bt2x_dp_align_dev(self.h, d_reads, d_quals, d_refs, d_in, n, d_out, d_recs,
                                       rec_cap, d_edits, edit_cap, d_counters, None, launch_flags, stream),
              "bt2x_dp_align_dev")

    def capabilities(self) -> int:
        """bt2x_capabilities: abi.CAP_* bits."""
        caps = ctypes.c_uint32(0)
        check(load().bt2x_capabilities(self.h, ctypes.byref(caps)), "bt2x_capabilities")
        return int(caps.value)

    def set_option(self, option: int, value: int) -> None:
        check(load().bt2x_set_option(self.h, option, int(value)), "bt2x_set_option")

    # ------------------------------------------------------- SA resolution
    def resolve(self, rows, qlen, reject_straddle: bool = False) -> np.ndarray:
        """BW rows (+ hit lengths) -> RESOLVE_OUT records: joined offset, reference
        index/offset/length, straddle flag (GroupWalk2S::advanceElement + joinedToTextOff)."""
        rows = np.asarray(rows, dtype=np.uint64)
        inp = np.zeros(len(rows), dtype=abi.RESOLVE_IN)
        inp["row"] = rows
        inp["qlen"] = qlen
        out = np.zeros(len(rows), dtype=abi.RESOLVE_OUT)
        check(load().bt2x_resolve(self.h, abi.ptr(inp), len(inp), int(reject_straddle), abi.ptr(out)),
              "bt2x_resolve")
        return out

    def resolve_dev(self, d_in: int, n: int, d_out: int, reject_straddle=False, stream=0):
        check(load().bt2x_resolve_dev(self.h, d_in, n, int(reject_straddle), d_out, stream),
              "bt2x_resolve_dev")

    # ------------------------------------------------------------ seed round
    def seed_round(self, reads, seeds, inp, exr, maxelt, sat_cap=None, elt_cap=None, exr_cap=None):
        """bt2x_seed_round (host buffers) -> (round_out, sats, elts, exr_out); arenas grown
        and the call repeated once on BT2X_E_OVERFLOW.  seeds = None: the GPU instantiates
        them (inp's seed0 / nseeds / seedflags)."""
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        inp = np.ascontiguousarray(inp, dtype=abi.ROUND_IN)
        gen = seeds is None
        nseeds = int((inp["seed0"] + inp["nseeds"]).max()) if gen and len(inp) else 0
        seeds = np.zeros(0, dtype=abi.SEED_IN) if gen else np.ascontiguousarray(seeds, dtype=abi.SEED_IN)
        exr = np.ascontiguousarray(exr if len(exr) else np.zeros(0, dtype=abi.EXRANGE), dtype=abi.EXRANGE)
        n = len(inp)
        sat_cap = sat_cap or 16 * n + 1024
        elt_cap = elt_cap or 64 * n + 1024
        exr_cap = exr_cap or 4 * n + 256
        out = np.zeros(n, dtype=abi.ROUND_OUT)
        sats = np.zeros(sat_cap, dtype=abi.SAT)
        elts = np.zeros(elt_cap, dtype=abi.ELT)
        exro = np.zeros(exr_cap, dtype=abi.EXRANGE)
        used = (ctypes.c_uint32 * 3)()
        rc = load().bt2x_seed_round(self.h, abi.ptr(reads), reads.nbytes, None if gen else abi.ptr(seeds),
                                    nseeds if gen else len(seeds), abi.ptr(inp), n,
                                    abi.ptr(exr), len(exr), maxelt, abi.ptr(out), abi.ptr(sats), sat_cap,
                                    abi.ptr(elts), elt_cap, abi.ptr(exro), exr_cap, used)
        if rc == abi.E_OVERFLOW:
            return self.seed_round(reads, None if gen else seeds, inp, exr, maxelt, max(sat_cap, used[0]), max(elt_cap, used[1]),
                                   max(exr_cap, used[2]))
        check(rc, "bt2x_seed_round")
        return out, sats[: used[0]], elts[: used[1]], exro[: used[2]]

    def seed_round_dev(self, d_reads, d_seeds, nseeds, d_in, nreads, d_exr, maxelt, d_out, d_sats, sat_cap,
                       d_elts, elt_cap, d_exr_out, exr_cap, d_used, stream=0):
        """bt2x_seed_round_dev: seed search + ranking/prioritization + SA resolution of a
        batch of reads, inputs resident in HBM.  d_used: 4 x u32 in HBM (arena use, then
        the count of reads whose GPU-instantiated seeds differ from nseeds)."""
        check(load().bt2x_seed_round_dev(self.h, d_reads, d_seeds, nseeds, d_in, nreads, d_exr, maxelt, d_out,
                                         d_sats, sat_cap, d_elts, elt_cap, d_exr_out, exr_cap, d_used, stream),
              "bt2x_seed_round_dev")

    def device_name(self) -> str:
        try:
            import torch
            return torch.cuda.get_device_name(0)
        except Exception:
            return "hip device"

    # ------------------------------------------------------------ metrics
    def last_kernel_ms(self, kernel: int) -> float:
        return float(load().bt2x_last_kernel_ms(self.h, kernel))

    def suffix_array(self, first: int = 0, n: int | None = None) -> np.ndarray:
        """Rows [first, first+n) of the device-resident full suffix array (uint32)."""
        if n is None:
            n = int(self.index.desc.len) + 1 - first
        out = np.zeros(n, dtype=np.uint32)
        check(load().bt2x_suffix_array(self.h, first, n, abi.ptr(out)), "bt2x_suffix_array")
        return out

    def last_counters(self, kernel: int) -> dict:
        c = abi.Counters()
        check(load().bt2x_last_counters(self.h, kernel, ctypes.byref(c)), "bt2x_last_counters")
        return c.as_dict()

    def last_round_stats(self) -> dict:
        """The last seed round's sampling work (bt2x_last_round_stats_ex)."""
        o = (ctypes.c_uint32 * 12)()
        rc = load().bt2x_last_round_stats_ex(self.h, o, 12)
        check(min(rc, 0), "bt2x_last_round_stats_ex")
        return {"reads": o[0], "jobs": o[1], "samples": o[2], "max_samples": o[3], "batches": o[4],
                "batch_draws": o[5], "serial_draws": o[6], "swap_draws": o[7], "kcyc_setup": o[8],
                "kcyc_batch": o[9], "kcyc_serial": o[10], "kcyc_rest": o[11]}


def build_index(fasta: str, outbase: str, off_rate: int = 4, ftab_chars: int = 10) -> str:
    """Write <outbase>.{1,2,3,4}.bt2l (bt2x_build_index); returns outbase."""
    check(load().bt2x_build_index(fasta.encode(), outbase.encode(), off_rate, ftab_chars),
          f"bt2x_build_index({fasta})")
    return outbase


def build_index_sa(fasta: str, outbase: str, sa, off_rate: int = 4, ftab_chars: int = 10,
                   bwt=None, keys=None) -> str:
    """bt2x_build_index_sa with a caller-sorted suffix array (uint64 numpy array, len+1)
    and optional per-row gathers bwt (uint8) / keys (uint32)."""
    import numpy as np
    sa = np.ascontiguousarray(sa, dtype=np.uint64)
    if bwt is not None:
        bwt = np.ascontiguousarray(bwt, dtype=np.uint8)
        assert len(bwt) == len(sa)
    if keys is not None:
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        assert len(keys) == len(sa)
    check(load().bt2x_build_index_sa(fasta.encode(), outbase.encode(), off_rate, ftab_chars,
                                     sa.ctypes.data, len(sa),
                                     None if bwt is None else bwt.ctypes.data,
                                     None if keys is None else keys.ctypes.data),
          f"bt2x_build_index_sa({fasta})")
    return outbase


def abi_sizes() -> list[int]:
    buf = (ctypes.c_uint32 * 32)()
    n = load().bt2x_abi_sizes(buf, 32)
    return list(buf[:min(n, 32)])
