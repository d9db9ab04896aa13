#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY: build oracle/_ref/bowtie2-align-l-bt2x, the reference aligner
with INTEGRATION.md's two patches applied -- its seed search and its SwAligner DP routed
through libbt2x.so (include/bt2x_ref_glue.hpp over include/bt2x_shims.hpp) -- so the
drop-in is executed, not only compiled (tests/test_integration.py runs it on the GPU
against the stock reference's SAM).

The reference is compiled as its Makefile does (one translation unit, bowtie2-align.cpp,
with oracle/Makefile's REFDEFS), from /root/reference where it lies.  The patch is made on
the *preprocessed* translation unit in a temporary directory outside the repository: the
bodies of six member functions are replaced by the glue calls below (brace matching is
exact there: no #ifdef branches left).  Nothing of the reference is written into the
repository; the only output is the binary in oracle/_ref/ (git-ignored).

  MultiSeedAligner::searchAllSeedsDoAll   aligner_seed.cpp:674-725
  SwAligner::initRead                     aligner_sw.cpp:35-59
  SwAligner::initRef (BitPairReference)   aligner_sw.cpp:117-229
  SwAligner::align                        aligner_sw.cpp:235-246
  SwAligner::nextAlignment                aligner_sw.cpp:252-375
  SwAligner::done                         aligner_sw.h:322-325

With --cpu the binary links oracle/bt2x_abi_oracle.cpp (the C-ABI answered by the CPU
oracle) instead of libbt2x.so, so the CPU suite runs the same glue; BT2X_GLUE_TRACE=1 at run
time prints one line per patched call.

    python3 oracle/ref_glue_build.py [--ref /root/reference] [--i16] [--cpu] [--only seeds|sw]
"""
from __future__ import annotations

import argparse
import os
import re
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIBDIR = os.path.join(ROOT, "omp-bowtie2-prime_amd", "bt2x")

REFDEFS = ["-DFORCE_ALL_OMP", "-DPOPCNT_CAPABILITY", "-DNO_SPINLOCK", "-DWITH_QUEUELOCK=1", "-D_LARGEFILE_SOURCE",
           "-D_FILE_OFFSET_BITS=64", "-D_GNU_SOURCE", "-DBOWTIE_MM", "-DBOWTIE2", "-DBOWTIE_64BIT_INDEX", "-DNDEBUG",
           '-DBOWTIE2_VERSION="2.5.4"', '-DBUILD_HOST="oracle"', '-DBUILD_TIME="oracle"', '-DCOMPILER_VERSION="g++"',
           '-DCOMPILER_OPTIONS="-O3 -msse2"']
CXXFLAGS = ["-O3", "-msse2", "-std=c++17", "-fopenmp", "-fno-strict-aliasing", "-w"]

WRAPPER = r'''
#include "bt2x_refglue.hpp"
#include "bowtie2-align.cpp"
namespace bt2x_refglue {
// one context per process: the reference's index prefix (-x) and scoring scheme, both set
// by its main before any worker thread runs; never closed (process exit tears HIP down)
bt2x::Device& device() {
	static bt2x::Device* d = [] {
		bt2x::Index* idx = new bt2x::Index(bt2index.c_str(), true);
		return new bt2x::Device(0, *idx, scoring_of(*multiseed_sc));
	}();
	return *d;
}
}
'''

# (signature regex, selector on the parameter text or None, new body)
PATCHES = [
    (r"void\s+MultiSeedAligner::searchAllSeedsDoAll\s*\(", None, r'''{
	std::lock_guard<std::mutex> g_(bt2x_refglue::gpu_mutex());
	static bt2x::MultiSeedAlignerHip* gpu_ = new bt2x::MultiSeedAlignerHip(bt2x_refglue::device());
	if(!bt2x::glue::search_all_seeds(*gpu_, _paramVec, _dataVec, _bufVec_filled, doExtend)) throw 1;
	if(bt2x_refglue::trace())
		for(size_t i_ = 0; i_ < _bufVec_filled; i_++)
			fprintf(stderr, "GLUE seed %zu fw=%d off=%d topf=%llu botf=%llu nlex=%u rep=%d\n", i_, (int)_paramVec[i_].fw,
			        (int)_paramVec[i_].sr->idx2off(_paramVec[i_].seedoffidx), (unsigned long long)_dataVec[i_].bwt.topf,
			        (unsigned long long)_dataVec[i_].bwt.botf, (unsigned)_dataVec[i_].nlex, (int)_dataVec[i_].need_reporting);
}'''),
    (r"bool\s+SwAligner::initRead\s*\(", None, r'''{
	rdfw_ = &rdfw; rdrc_ = &rdrc; qufw_ = &qufw; qurc_ = &qurc; rdlen_ = rdlen; sc_ = &sc;
	nceil_ = sc.nCeil.f<int>((double)rdfw.length());
	initedRead_ = bt2x_refglue::sw(this).swa.initRead(rdfw, rdrc, qufw, qurc, rdlen, sc);
	return initedRead_;
}'''),
    (r"bool\s+SwAligner::initRef\s*\(", "BitPairReference", r'''{
	bt2x_refglue::Sw& s_ = bt2x_refglue::sw(this);
	s_.refidx = (size_t)refidx; s_.reflen = (int64_t)reflen;
	fw_ = fw;
	initedRef_ = s_.swa.initRef(fw, (size_t)refidx, rect, refs, (int64_t)reflen, (int64_t)minsc, enable8, extend, upto, nsUpto);
	if(bt2x_refglue::trace())
		fprintf(stderr, "GLUE initRef fw=%d ref=%zu rect=[%lld,%lld] minsc=%lld ok=%d\n", (int)fw, (size_t)refidx,
		        (long long)rect.refl, (long long)rect.refr, (long long)minsc, (int)initedRef_);
	return initedRef_;
}'''),
    (r"bool\s+SwAligner::align\s*\(", None, r'''{
	std::lock_guard<std::mutex> g_(bt2x_refglue::gpu_mutex());
	int64_t b_ = 0;
	const bool ok_ = bt2x_refglue::sw(this).swa.align(b_);
	best = (TAlScore)b_;
	if(bt2x_refglue::trace()) fprintf(stderr, "GLUE align ok=%d best=%lld\n", (int)ok_, (long long)b_);
	return ok_;
}'''),
    (r"bool\s+SwAligner::nextAlignment\s*\(", None, r'''{
	bt2x_refglue::Sw& s_ = bt2x_refglue::sw(this);
	bt2x::AlnView v_;
	const bool ok_ = s_.swa.nextAlignment(v_, (int64_t)minsc, rnd);
	bt2x::glue::to_swresult(v_, ok_, res, s_.refidx, s_.reflen, rdlen_);
	if(bt2x_refglue::trace())
		fprintf(stderr, "GLUE next ok=%d score=%lld refoff=%lld fw=%d ned=%zu\n", (int)ok_, (long long)v_.score,
		        (long long)v_.refoff, (int)v_.fw, (size_t)v_.edits.size());
	return ok_;
}'''),
]


def skip_string(s: str, i: int) -> int:
    q = s[i]
    i += 1
    while s[i] != q:
        i += 2 if s[i] == "\\" else 1
    return i + 1


def match_brace(s: str, i: int) -> int:
    """s[i] == '{': index just past its matching '}' (string and char literals skipped;
    a preprocessed unit has no comments)."""
    depth = 0
    while True:
        c = s[i]
        if c in "\"'":
            i = skip_string(s, i)
            continue
        if c == "{":
            depth += 1
        elif c == "}":
            depth -= 1
            if depth == 0:
                return i + 1
        i += 1


def replace_body(src: str, sig: str, select: str | None, body: str, start: int = 0) -> str:
    for m in re.finditer(sig, src[start:]):
        a = start + m.end()
        # the parameter list: to the matching ')'
        depth, j = 1, a
        while depth:
            depth += {"(": 1, ")": -1}.get(src[j], 0)
            j += 1
        params = src[a:j]
        k = j
        while src[k] in " \t\r\n":
            k += 1
        if src[k] == ";":                         # a declaration
            continue
        if src[k:k + 5] == "const":
            k += 5
            while src[k] in " \t\r\n":
                k += 1
        if src[k] != "{" or (select and select not in params):
            continue
        e = match_brace(src, k)
        return src[:k] + body + src[e:]
    raise SystemExit(f"ref_glue_build: no definition matches {sig} {select or ''}")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--i16", action="store_true", help="the -DENABLE_I16 build")
    ap.add_argument("--cpu", action="store_true",
                    help="link oracle/bt2x_abi_oracle.cpp (the C-ABI answered by the CPU oracle) instead of "
                         "libbt2x.so, so the patched aligner runs in the CPU test suite")
    ap.add_argument("--only", choices=["seeds", "sw"], default=None,
                    help="apply only the seed-search or only the SwAligner patch (bisecting a mismatch)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    out = a.out or os.path.join(HERE, "_ref", "bowtie2-align-l-bt2x" + ("-i16" if a.i16 else "") +
                                ("-cpu" if a.cpu else ""))
    os.makedirs(os.path.dirname(out), exist_ok=True)
    deps = [os.path.abspath(__file__), os.path.join(HERE, "bt2x_refglue.hpp")] + \
        [os.path.join(ROOT, "include", h) for h in ("bt2x.h", "bt2x_shims.hpp", "bt2x_ref_glue.hpp")] + \
        ([os.path.join(HERE, f) for f in ("bt2x_abi_oracle.cpp", "bt2x_oracle.c", "bt2x_oracle.h")] if a.cpu else [])
    if os.path.exists(out) and os.path.getmtime(out) > max(os.path.getmtime(d) for d in deps):
        return                                    # up to date (libbt2x.so is linked dynamically)
    cxx = os.environ.get("CXX", "g++")
    tmp = tempfile.mkdtemp(prefix="bt2x_refglue_")
    try:
        tu = os.path.join(tmp, "glue_tu.cpp")
        with open(tu, "w") as f:
            f.write(WRAPPER)
        defs = REFDEFS + (["-DENABLE_I16"] if a.i16 else [])
        ii = os.path.join(tmp, "glue_tu.ii")
        subprocess.run([cxx, "-E", "-P"] + CXXFLAGS + defs + ["-I" + a.ref, "-I" + os.path.join(a.ref, "third_party"),
                        "-I" + os.path.join(ROOT, "include"), "-I" + HERE, tu, "-o", ii], check=True)
        src = open(ii).read()
        for sig, sel, body in PATCHES:
            if a.only and (a.only == "seeds") != ("searchAllSeeds" in sig):
                continue
            src = replace_body(src, sig, sel, body)
        # SwAligner::done(), an inline member in the class body
        c = None if a.only == "seeds" else re.search(r"class\s+SwAligner\s*\{", src)
        if not c and a.only != "seeds":
            raise SystemExit("ref_glue_build: class SwAligner not found")
        if c:
            src = replace_body(src, r"bool\s+done\s*\(", None, r'''{
		return bt2x_refglue::sw(this).swa.done();
	}''', start=c.end())
        with open(ii, "w") as f:
            f.write(src)
        if a.cpu:
            objs = [os.path.join(tmp, "abi.o"), os.path.join(tmp, "oracle.o")]
            subprocess.run([cxx, "-O2", "-std=c++17", "-c", os.path.join(HERE, "bt2x_abi_oracle.cpp"), "-I" + HERE,
                            "-o", objs[0]], check=True)
            subprocess.run([os.environ.get("CC", "gcc"), "-O2", "-std=c11", "-ffp-contract=off", "-c",
                            os.path.join(HERE, "bt2x_oracle.c"), "-o", objs[1]], check=True)
            link = ["-x", "none"] + objs
        else:
            link = ["-L" + LIBDIR, "-lbt2x", "-Wl,-rpath,$ORIGIN/../../omp-bowtie2-prime_amd/bt2x", "-L/opt/rocm/lib",
                    "-Wl,-rpath,/opt/rocm/lib"]
        subprocess.run([cxx] + CXXFLAGS + ["-x", "c++", ii, "-o", out] + link + ["-lpthread", "-lz"], check=True)
        print(f"ref_glue_build: {out}", file=sys.stderr)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
