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


def main() -> None:
    run(["make", "-C", os.path.join(ROOT, "oracle"), "ref", "oracle"])
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
