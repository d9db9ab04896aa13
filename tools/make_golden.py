#!/usr/bin/env python3
"""Regenerate tests/golden/ from the reference itself (run in the dev container,
where /root/reference exists; never on the GPU box).

Steps (all outputs xz-compressed under tests/golden/):
  1. make -C oracle ref          -> oracle/_ref/{bowtie2-build-l,refharness}
  2. lambda: index built by the reference's bowtie2-build-l from
     example/reference/lambda_virus.fa; reads = first 2000 records of the shipped
     example/reads/longreads.fq; seeds golden = refharness seeds.
  3. rep: seeded synthetic 300 kbp genome with repeat families / low complexity / N
     runs (tools/simdata.py), reference-built index, simulated reads of several
     lengths (and an N-rich set); seeds golden + DP golden at the reference defaults,
     DP golden at --dpad 12 (config C3's setting) and DP golden under a non-default
     scoring scheme.
  4. resolve: the committed lambda and rep indexes/reads through refharness resolve
     (GroupWalk2S + joinedToTextOff on every reported seed range, fragment-boundary
     probes) and, for rep, refharness rank (searchAllSeedsFinalize + rankSeedHits).
     `make_golden.py resolve` regenerates only these.
  5. e2e: the reference aligner (bowtie2-align-l, 1 thread) on the lambda and rep
     fixtures, default and --dpad 12 / non-default scoring, as sorted @PG-less SAM.
     `make_golden.py e2e` regenerates only these.
  6. i16 (`make_golden.py i16`): the -DENABLE_I16 reference builds (refharness-i16,
     bowtie2-align-l-i16) -- DP vectors and SAM of the signed 16-bit kernel (--no-sse8).
  7. md5 (`make_golden.py md5`): e2e_md5.json, md5s of sets too large to commit as SAM
  8. summary (`make_golden.py summary`): e2e_summary.json, the reference's alignment
     summary (ReportingMetrics) for the e2e and md5 sets
     (config C2's E. coli stand-in, 50k-read lane-kernel launches, all of config C1).
Each text golden file starts with a '#' header naming the command that produced it.
"""
from __future__ import annotations

import lzma
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = os.environ.get("BT2X_REFERENCE", "/root/reference")
GOLD = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, HERE)
import simdata as sd  # noqa: E402

BUILD = os.path.join(ROOT, "oracle", "_ref", "bowtie2-build-l")
HARN = os.path.join(ROOT, "oracle", "_ref", "refharness")

# non-default scoring variant used by dp_rep_alt (must match tests/test_oracle_golden.py)
ALT_OPTS = ["--mp", "5,1", "--np", "2", "--rdg", "4,2", "--rfg", "6,3", "--gbar", "2"]


def xz_copy(src: str, dst: str) -> None:
    with open(src, "rb") as fi, lzma.open(dst, "wb", preset=9 | lzma.PRESET_EXTREME) as fo:
        shutil.copyfileobj(fi, fo)


def run(cmd, **kw):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, **kw)


def xz_unpack(src: str, dst: str) -> None:
    with lzma.open(src, "rb") as fi, open(dst, "wb") as fo:
        shutil.copyfileobj(fi, fo)


def resolve_goldens(tmp: str) -> None:
    for name, fq in (("lambda_virus", "lambda_longreads.fq"), ("rep", "rep_reads.fq")):
        base = os.path.join(tmp, name)
        for k in "1234":
            xz_unpack(os.path.join(GOLD, f"{name}.{k}.bt2l.xz"), f"{base}.{k}.bt2l")
        rfq = os.path.join(tmp, fq)
        xz_unpack(os.path.join(GOLD, fq + ".xz"), rfq)
        tag = "lambda" if name == "lambda_virus" else name
        out = os.path.join(tmp, f"resolve_{tag}.txt")
        run([HARN, "resolve", base, rfq, out])
        xz_copy(out, os.path.join(GOLD, f"resolve_{tag}.txt.xz"))
        if name == "rep":
            out = os.path.join(tmp, "rank_rep.txt")
            run([HARN, "rank", base, rfq, out])
            xz_copy(out, os.path.join(GOLD, "rank_rep.txt.xz"))


ALIGN = os.path.join(ROOT, "oracle", "_ref", "bowtie2-align-l")

# end-to-end SAM goldens: (name, index, reads fixture, extra bowtie2-align-l options)
E2E_SETS = [("e2e_lambda", "lambda_virus", "lambda_longreads.fq", []),
            ("e2e_rep", "rep", "rep_reads.fq", []),
            ("e2e_rep_dpad12", "rep", "rep_reads.fq", ["--dpad", "12"]),
            ("e2e_rep_alt", "rep", "rep_reads.fq", ALT_OPTS)]


def sam_records(path: str) -> bytes:
    """SAM minus @PG, records sorted: the reference's own comparison methodology
    (scripts/sim Sim.pm: sort, strip @PG), which is also independent of how reads
    finish across seed rounds."""
    with open(path, "rb") as f:
        lines = [ln for ln in f.read().split(b"\n") if ln and not ln.startswith(b"@PG")]
    hdr = [ln for ln in lines if ln.startswith(b"@")]
    rec = sorted(ln for ln in lines if not ln.startswith(b"@"))
    return b"\n".join(hdr + rec) + b"\n"


def e2e_goldens(tmp: str) -> None:
    """The reference aligner itself (OMP_NUM_THREADS=1) on the committed fixtures."""
    for name, idx, fq, opts in E2E_SETS:
        base = os.path.join(tmp, idx)
        if not os.path.exists(base + ".4.bt2l"):
            for k in "1234":
                xz_unpack(os.path.join(GOLD, f"{idx}.{k}.bt2l.xz"), f"{base}.{k}.bt2l")
        rfq = os.path.join(tmp, fq)
        if not os.path.exists(rfq):
            xz_unpack(os.path.join(GOLD, fq + ".xz"), rfq)
        sam = os.path.join(tmp, name + ".sam")
        env = dict(os.environ, OMP_NUM_THREADS="1")
        run([ALIGN, "-x", base, "-U", rfq, "-S", sam] + opts, env=env, stderr=subprocess.DEVNULL)
        with lzma.open(os.path.join(GOLD, name + ".sam.xz"), "wb", preset=9 | lzma.PRESET_EXTREME) as fo:
            fo.write(sam_records(sam))


TANDEM_SETS = [("e2e_tandem", []), ("e2e_tandem_dpad12", ["--dpad", "12"])]


def tandem_goldens(tmp: str) -> None:
    """Tandem-repeat fixture: reads whose DP windows hold several alignments, so -M's
    score tightening (aligner_sw_driver.cpp:589-619) happens between nextAlignment calls
    of one DP problem.  Index by the reference builder, SAM by the reference aligner."""
    g, arrays = sd.gen_tandem_genome(nchrom=4, chrom_len=40000, arrays_per_chrom=12, seed=21)
    fa = os.path.join(tmp, "tandem.fa")
    sd.write_fasta(fa, g)
    base = os.path.join(tmp, "tandem")
    run([BUILD, fa, base], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    for k in "1234":
        xz_copy(f"{base}.{k}.bt2l", os.path.join(GOLD, f"tandem.{k}.bt2l.xz"))
    reads = (sd.sim_reads_in(g, arrays, 1200, 100, seed=31) + sd.sim_reads_in(g, arrays, 800, 150, seed=32)
             + sd.sim_reads_in(g, arrays, 300, 60, seed=33, sub_rate=0.03))
    rfq = os.path.join(tmp, "tandem_reads.fq")
    sd.write_fastq(rfq, reads)
    xz_copy(rfq, os.path.join(GOLD, "tandem_reads.fq.xz"))
    for name, opts in TANDEM_SETS:
        sam = os.path.join(tmp, name + ".sam")
        env = dict(os.environ, OMP_NUM_THREADS="1")
        run([ALIGN, "-x", base, "-U", rfq, "-S", sam] + opts, env=env, stderr=subprocess.DEVNULL)
        with lzma.open(os.path.join(GOLD, name + ".sam.xz"), "wb", preset=9 | lzma.PRESET_EXTREME) as fo:
            fo.write(sam_records(sam))


ALIGN16 = os.path.join(ROOT, "oracle", "_ref", "bowtie2-align-l-i16")
HARN16 = os.path.join(ROOT, "oracle", "_ref", "refharness-i16")
WIDE_MIN = ["--score-min", "L,-0.6,-2.5", "--dpad", "12"]   # minsc below -254 from 102 bp on

# the i16 DP (BASELINE config C2): -DENABLE_I16 reference builds.  dp: the
# refharness dp set over the rep reads with --no-sse8, with a minimum score below the u8
# floor, and the i16 build's default (u8 unless minsc < -254: mixed launches)
I16_DP_SETS = [("dp_rep_i16", "1234", ["--no-sse8"]),
               ("dp_rep_i16_wide", "99", ["--no-sse8"] + WIDE_MIN),
               ("dp_rep_i16_mix", "77", WIDE_MIN)]
I16_E2E_SETS = [("e2e_rep_i16", "rep", "rep_reads.fq", ["--no-sse8"]),
                ("e2e_tandem_i16", "tandem", "tandem_reads.fq", ["--no-sse8"]),
                ("e2e_rep_i16_wide", "rep", "rep_reads.fq", ["--no-sse8"] + WIDE_MIN),
                ("e2e_rep_i16_mix", "rep", "rep_reads.fq", WIDE_MIN)]


def i16_goldens(tmp: str) -> None:
    """DP vectors and SAM of the reference's i16 kernel (refharness-i16, bowtie2-align-l-i16)."""
    for idx in ("rep", "tandem"):
        base = os.path.join(tmp, idx)
        for k in "1234":
            xz_unpack(os.path.join(GOLD, f"{idx}.{k}.bt2l.xz"), f"{base}.{k}.bt2l")
    for fq in ("rep_reads.fq", "tandem_reads.fq"):
        xz_unpack(os.path.join(GOLD, fq + ".xz"), os.path.join(tmp, fq))
    rep, rfq = os.path.join(tmp, "rep"), os.path.join(tmp, "rep_reads.fq")
    # the wide/mixed DP sets use reads 1450..1899 (100 and 150 bp: minsc on both sides of -254)
    sub = os.path.join(tmp, "rep_reads_sub.fq")
    with open(rfq) as fi, open(sub, "w") as fo:
        for i, line in enumerate(fi):
            if 4 * 1450 <= i < 4 * 1900:
                fo.write(line)
    for name, seed, opts in I16_DP_SETS:
        out = os.path.join(tmp, name + ".txt")
        run([HARN16, "dp", rep, rfq if name == "dp_rep_i16" else sub, out, seed] + opts)
        xz_copy(out, os.path.join(GOLD, name + ".txt.xz"))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for name, idx, fq, opts in I16_E2E_SETS:
        sam = os.path.join(tmp, name + ".sam")
        run([ALIGN16, "-x", os.path.join(tmp, idx), "-U", os.path.join(tmp, fq), "-S", sam] + opts,
            env=env, stderr=subprocess.DEVNULL)
        with lzma.open(os.path.join(GOLD, name + ".sam.xz"), "wb", preset=9 | lzma.PRESET_EXTREME) as fo:
            fo.write(sam_records(sam))


# md5 goldens (tests/golden/e2e_md5.json): sets too large to commit as SAM.  md5 of the
# sorted records minus @PG (`grep -v '^@PG' | sort | md5sum`, SURVEY.md:508's procedure).
#   ecoli_*: config C2 -- the seeded 4.64 Mbp genome (simdata.ecoli_genome, indexed by the
#            reference builder; FASTA and index md5s pinned) with simdata.fixture_reads
#   ecoli_large_*: 50k x 150 bp at --dpad 12: DP launches of > 32k problems (the lane kernel)
#   ecoli_c5_400: config C5's read shape, 20k fixed-length 400 bp reads: every read is
#            unaligned (rdlen >= 256, bt2_search.cpp:2475-2496)
#   ecoli_long_200: 200 bp reads (161..255: seeded, then initRead's 160-row cap, F2)
#   lambda_full: config C1, all 6000 example/reads/longreads.fq reads, 1 thread
MD5_SETS = [("ecoli_i16", 10000, 100, 1, "i16", ["--no-sse8"]),
            ("ecoli_u8", 10000, 100, 1, "u8", []),
            ("ecoli_large_u8", 50000, 150, 3, "u8", ["--dpad", "12"]),
            ("ecoli_large_i16", 50000, 150, 3, "i16", ["--no-sse8", "--dpad", "12"]),
            ("ecoli_c5_400", 20000, 400, 5, "u8", []),
            ("ecoli_long_200", 4000, 200, 5, "u8", [])]


def sam_md5(path: str) -> tuple[str, int, int]:
    import hashlib
    with open(path, "rb") as f:
        lines = [ln for ln in f.read().split(b"\n") if ln and not ln.startswith(b"@PG")]
    recs = [ln for ln in lines if not ln.startswith(b"@")]
    aligned = sum(1 for ln in recs if ln.split(b"\t")[1] != b"4")
    data = b"".join(ln + b"\n" for ln in sorted(lines))
    return hashlib.md5(data).hexdigest(), len(recs), aligned


def md5_goldens(tmp: str) -> None:
    import hashlib
    import json
    g = sd.ecoli_genome()
    fa = os.path.join(tmp, "ecoli.fa")
    sd.write_fasta(fa, g)
    base = os.path.join(tmp, "ecoli")
    run([BUILD, fa, base], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    md5 = lambda p: hashlib.md5(open(p, "rb").read()).hexdigest()     # noqa: E731
    out = {"_note": "tools/make_golden.py md5: sorted SAM records minus @PG of the reference aligner "
                    "(1 thread); genome/reads from tools/simdata.py",
           "ecoli_fasta_md5": md5(fa), "ecoli_index_md5": {k: md5(f"{base}.{k}.bt2l") for k in "1234"},
           "sets": {}}
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for name, n, rdlen, seed, binary, opts in MD5_SETS:
        fq = os.path.join(tmp, f"{name}.fq")
        sd.fixture_reads(g, fq, n, rdlen, seed)
        sam = os.path.join(tmp, name + ".sam")
        run([ALIGN16 if binary == "i16" else ALIGN, "-x", base, "-U", fq, "-S", sam] + opts,
            env=env, stderr=subprocess.DEVNULL)
        h, nrec, nal = sam_md5(sam)
        out["sets"][name] = {"genome": "ecoli", "reads": n, "read_len": rdlen, "seed": seed, "binary": binary,
                             "opts": opts, "md5": h, "records": nrec, "aligned": nal}
    # C1: the shipped lambda example, every read
    lam = os.path.join(tmp, "lambda_virus")
    for k in "1234":
        xz_unpack(os.path.join(GOLD, f"lambda_virus.{k}.bt2l.xz"), f"{lam}.{k}.bt2l")
    sam = os.path.join(tmp, "lambda_full.sam")
    run([ALIGN, "-x", lam, "-U", os.path.join(REF, "example/reads/longreads.fq"), "-S", sam],
        env=env, stderr=subprocess.DEVNULL)
    h, nrec, nal = sam_md5(sam)
    out["sets"]["lambda_full"] = {"genome": "lambda_virus", "reads": nrec, "fastq": "lambda_longreads_full.fq.xz",
                                  "binary": "u8", "opts": [], "md5": h, "records": nrec, "aligned": nal}
    xz_copy(os.path.join(REF, "example/reads/longreads.fq"), os.path.join(GOLD, "lambda_longreads_full.fq.xz"))
    with open(os.path.join(GOLD, "e2e_md5.json"), "w") as f:
        json.dump(out, f, indent=1)


def ref_summary(stderr: str) -> str:
    """The reference's alignment summary (AlnSink::printAlSumm) from its stderr, without
    the Timer: lines it prints alongside (bt2_search.cpp MyTimer dump)."""
    return "".join(ln + "\n" for ln in stderr.splitlines() if ln and not ln.startswith("Timer:"))


def summary_goldens(tmp: str) -> None:
    """e2e_summary.json: the reference's alignment summary for the committed e2e sets and
    the E. coli md5 sets (the metrics bt2x-align --metrics and bt2x.dist reproduce)."""
    import json
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = {"_note": "tools/make_golden.py summary: the reference aligner's stderr summary (1 thread)", "sets": {}}
    sets = ([(n, i, f, o, ALIGN) for n, i, f, o in E2E_SETS] +
            [(n, "tandem", "tandem_reads.fq", o, ALIGN) for n, o in TANDEM_SETS] +
            [(n, i, f, o, ALIGN16) for n, i, f, o in I16_E2E_SETS])
    for name, idx, fq, opts, binary in sets:
        base = os.path.join(tmp, idx)
        if not os.path.exists(base + ".4.bt2l"):
            for k in "1234":
                xz_unpack(os.path.join(GOLD, f"{idx}.{k}.bt2l.xz"), f"{base}.{k}.bt2l")
        rfq = os.path.join(tmp, fq)
        if not os.path.exists(rfq):
            xz_unpack(os.path.join(GOLD, fq + ".xz"), rfq)
        r = subprocess.run([binary, "-x", base, "-U", rfq, "-S", os.devnull] + opts, env=env, check=True,
                           capture_output=True, text=True)
        out["sets"][name] = {"index": idx, "fastq": fq + ".xz", "opts": opts,
                             "binary": "i16" if binary == ALIGN16 else "u8", "summary": ref_summary(r.stderr)}
    g = sd.ecoli_genome()
    fa = os.path.join(tmp, "ecoli.fa")
    sd.write_fasta(fa, g)
    base = os.path.join(tmp, "ecoli")
    run([BUILD, fa, base], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    for name, n, rdlen, seed, binary, opts in MD5_SETS:
        fq = os.path.join(tmp, f"{name}.fq")
        sd.fixture_reads(g, fq, n, rdlen, seed)
        r = subprocess.run([ALIGN16 if binary == "i16" else ALIGN, "-x", base, "-U", fq, "-S", os.devnull] + opts,
                           env=env, check=True, capture_output=True, text=True)
        out["sets"][name] = {"index": "ecoli", "reads": n, "read_len": rdlen, "seed": seed, "binary": binary,
                             "opts": opts, "summary": ref_summary(r.stderr)}
    with open(os.path.join(GOLD, "e2e_summary.json"), "w") as f:
        json.dump(out, f, indent=1)


def main() -> None:
    run(["make", "-C", os.path.join(ROOT, "oracle"), "ref", "oracle"])
    for cmd, fn in (("i16", i16_goldens), ("md5", md5_goldens), ("summary", summary_goldens)):
        if sys.argv[1:] == [cmd]:
            tmp = tempfile.mkdtemp(prefix="bt2x_golden_")
            try:
                fn(tmp)
            finally:
                shutil.rmtree(tmp, ignore_errors=True)
            return
    if sys.argv[1:] == ["tandem"]:
        tmp = tempfile.mkdtemp(prefix="bt2x_golden_")
        try:
            tandem_goldens(tmp)
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
        return
    if sys.argv[1:] == ["e2e"]:
        tmp = tempfile.mkdtemp(prefix="bt2x_golden_")
        try:
            e2e_goldens(tmp)
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
        return
    if sys.argv[1:] == ["resolve"]:
        tmp = tempfile.mkdtemp(prefix="bt2x_golden_")
        try:
            resolve_goldens(tmp)
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
        return
    os.makedirs(GOLD, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix="bt2x_golden_")
    try:
        # ---------------- lambda (the reference's own example data)
        lam = os.path.join(tmp, "lambda_virus")
        run([BUILD, os.path.join(REF, "example/reference/lambda_virus.fa"), lam],
            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        for k in "1234":
            xz_copy(f"{lam}.{k}.bt2l", os.path.join(GOLD, f"lambda_virus.{k}.bt2l.xz"))
        fq = os.path.join(tmp, "lambda_longreads.fq")
        with open(os.path.join(REF, "example/reads/longreads.fq")) as fi, open(fq, "w") as fo:
            for i, line in enumerate(fi):
                if i >= 4 * 2000:
                    break
                fo.write(line)
        xz_copy(fq, os.path.join(GOLD, "lambda_longreads.fq.xz"))
        out = os.path.join(tmp, "seeds_lambda.txt")
        run([HARN, "seeds", lam, fq, out])
        xz_copy(out, os.path.join(GOLD, "seeds_lambda.txt.xz"))

        # ---------------- rep (synthetic, repeat-rich)
        g = sd.gen_genome(300000, nchrom=3, seed=7, repeat_frac=0.3, n_runs_per_mb=20,
                          lowcomp_per_mb=40)
        fa = os.path.join(tmp, "rep.fa")
        sd.write_fasta(fa, g)
        rep = os.path.join(tmp, "rep")
        run([BUILD, fa, rep], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        for k in "1234":
            xz_copy(f"{rep}.{k}.bt2l", os.path.join(GOLD, f"rep.{k}.bt2l.xz"))
        xz_copy(fa, os.path.join(GOLD, "rep.fa.xz"))
        reads = (sd.sim_reads(g, 1500, 100, seed=11) + sd.sim_reads(g, 1000, 150, seed=12)
                 + sd.sim_reads(g, 300, 40, seed=13)
                 + sd.sim_reads(g, 200, 160, seed=14, allow_ref_n=True)
                 + sd.sim_reads(g, 100, 20, seed=15)
                 + sd.sim_reads(g, 300, 100, seed=16, n_rate=0.03, sub_rate=0.03)
                 + sd.sim_reads(g, 100, 139, seed=17) + sd.sim_reads(g, 60, 12, seed=18))
        rfq = os.path.join(tmp, "rep_reads.fq")
        sd.write_fastq(rfq, reads)
        xz_copy(rfq, os.path.join(GOLD, "rep_reads.fq.xz"))
        out = os.path.join(tmp, "seeds_rep.txt")
        run([HARN, "seeds", rep, rfq, out])
        xz_copy(out, os.path.join(GOLD, "seeds_rep.txt.xz"))
        for name, opts in (("dp_rep", []), ("dp_rep_dpad12", ["--dpad", "12"]),
                           ("dp_rep_alt", ALT_OPTS)):
            out = os.path.join(tmp, name + ".txt")
            run([HARN, "dp", rep, rfq, out, "1234"] + opts)
            xz_copy(out, os.path.join(GOLD, name + ".txt.xz"))
        # ---------------- builder known answers: tricky FASTA (empty/all-N/unnamed records,
        # IUPAC, lowercase, gaps) indexed by the reference builder
        import hashlib
        import json
        tri = os.path.join(GOLD, "tricky.fa")
        tb = os.path.join(tmp, "tricky")
        run([BUILD, tri, tb], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        md5 = {k: hashlib.md5(open(f"{tb}.{k}.bt2l", "rb").read()).hexdigest() for k in "1234"}
        with open(os.path.join(GOLD, "builder_md5.json"), "w") as f:
            json.dump({"tricky": md5, "_note": "md5 of oracle/_ref/bowtie2-build-l tests/golden/tricky.fa "
                       "output (tools/make_golden.py)"}, f, indent=1)
        resolve_goldens(tmp)
        e2e_goldens(tmp)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    for f in sorted(os.listdir(GOLD)):
        print(f"{os.path.getsize(os.path.join(GOLD, f)):>10}  {f}")


if __name__ == "__main__":
    main()
