"""CPU-side checks of the C-ABI boundary: the product library loads, exports every
entry point include/bt2x.h declares, its struct sizes match the numpy mirrors, the
host-side index loader agrees with the oracle's, and there is no CPU fallback."""
import ctypes
import os
import re

import numpy as np
import pytest

import golden_io as g
import oracle_lib as ol
from bt2x import abi, lib

HEADER = os.path.join(g.ROOT, "include", "bt2x.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = set(re.findall(r"\b(bt2x_[a-z0-9_]+)\s*\(", txt))
    inline = set(re.findall(r"static inline [^(;]*?\b(bt2x_[a-z0-9_]+)\s*\(", txt))   # header-only helpers
    return sorted(names - inline)


def test_library_exports_every_declared_symbol():
    L = lib.load()
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing
    assert set(declared_functions()) <= set(lib.FUNCS)


def test_struct_sizes_match_numpy_mirrors():
    s = lib.abi_sizes()
    assert s[:5] == [abi.SEED_IN.itemsize, abi.SEED_OUT.itemsize, abi.DP_IN.itemsize,
                     abi.DP_OUT.itemsize, abi.ALN_REC.itemsize]
    assert s[5] == ctypes.sizeof(abi.Scoring)
    assert s[6] == ctypes.sizeof(abi.IndexDesc)
    assert s[7] == ctypes.sizeof(abi.Counters)
    assert s[8:10] == [abi.RESOLVE_IN.itemsize, abi.RESOLVE_OUT.itemsize]
    assert s[10:14] == [abi.ROUND_IN.itemsize, abi.ROUND_OUT.itemsize, abi.SAT.itemsize, abi.EXRANGE.itemsize]
    assert s[14] == abi.ELT.itemsize == 8
    assert s[15] == abi.STORE_IN.itemsize == 16
    assert s[16] == abi.SAM_REQ.itemsize == 80


def test_scoring_tables_match_oracle():
    a, b = lib.default_scoring(), ol.default_scoring()
    assert list(a.mmpens) == list(b.mmpens) and list(a.npens) == list(b.npens)
    assert a.mmpens[0] == 2 and a.mmpens[40] == 6 and a.mmpens[30] == 5   # scoring.h:118-123
    c = lib.default_scoring(mm_max=5, mm_min=1)
    assert c.mmpens[40] == 5 and c.mmpens[0] == 1


@pytest.mark.parametrize("name", ["lambda_virus", "rep"])
def test_index_loader_matches_oracle_loader(golden_dir, name):
    base = g.materialize_index(name, str(golden_dir))
    a = lib.Index(base, load_offs=True)
    b = ol.OracleIndex(base, load_offs=True)
    for f in ("len", "zoff", "ftab_chars", "off_rate", "line_rate", "ebwt_bytes", "ftab_len",
              "eftab_len", "offs_len", "npat", "nfrag"):
        assert getattr(a.desc, f) == getattr(b.desc, f), f
    assert list(a.desc.fchr) == list(b.desc.fchr)
    np.testing.assert_array_equal(a.desc.array("ebwt", np.uint8, "ebwt_bytes"),
                                  b.desc.array("ebwt", np.uint8, "ebwt_bytes"))
    for arr, cnt in (("ftab", "ftab_len"), ("eftab", "eftab_len"), ("offs", "offs_len"),
                     ("plen", "npat")):
        np.testing.assert_array_equal(a.desc.array(arr, np.uint64, cnt), b.desc.array(arr, np.uint64, cnt))
    # fchr[4] is the text length and the last ftab entry is len+1 (bt2_idx.h:3180-3214)
    assert a.desc.fchr[4] == a.desc.len
    ftab = a.desc.array("ftab", np.uint64, "ftab_len")
    eftab = a.desc.array("eftab", np.uint64, "eftab_len")
    last = int(ftab[-1])
    hi = last if last <= a.desc.len else int(eftab[(last ^ 0xFFFFFFFFFFFFFFFF) * 2 + 1])
    assert hi == a.desc.len + 1


def test_missing_index_is_an_error():
    with pytest.raises(lib.Bt2xError):
        lib.Index("/nonexistent/index")


def test_no_cpu_fallback_without_gpu(golden_dir):
    """The product path fails loudly without a HIP device instead of computing on CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    base = g.materialize_index("lambda_virus", str(golden_dir))
    with pytest.raises(lib.Bt2xError):
        lib.Context(lib.Index(base))


def test_cpp_shim_binary_links_and_runs_without_gpu_work():
    """include/bt2x_shims.hpp compiles against bt2x.h and the test binary resolves
    libbt2x.so (usage path only: no device call)."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "test_shims")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.dirname(exe)], check=True, capture_output=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage" in r.stderr


def test_open_rejects_penalties_the_u8_kernel_cannot_pack(golden_dir):
    """--mp MX > 15 / --np > 15 are refused up front (BT2X_E_ARG), before any device
    work; the u8 DP kernel packs a row's penalty into 4 bits."""
    base = g.materialize_index("lambda_virus", str(golden_dir))
    idx = lib.Index(base)
    for kw in ({"mm_max": 16, "mm_min": 2}, {"n_pen": 16}):
        with pytest.raises(lib.Bt2xError) as e:
            lib.Context(idx, scoring=lib.default_scoring(**kw))
        assert e.value.code == abi.E_ARG
