#!/usr/bin/env python3
"""Host-driver timing without a GPU (development tool).

Builds (once, cached under /tmp/bt2x_hostprof) a seeded synthetic genome index and a
FASTQ of simulated 150 bp reads with bench.py's generator, then runs
tests/cpp/test_e2e_oracle --host-timing: a first pass records every kernel result
(CPU oracle), a second pass replays them, so the second pass's wall time is the host
driver alone (FASTQ parse, per-read logic, gathers/scatters, SAM formatting).

    python tools/host_profile.py [--mb 32] [--reads 200000] [-p 8] [--slots N] [extra args]
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omp-bowtie2-prime_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=32.0)
    ap.add_argument("--reads", type=int, default=200000)
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("-p", type=int, default=8)
    ap.add_argument("--slots", type=int, default=65536)
    ap.add_argument("--dpad", type=int, default=12)
    ap.add_argument("--check", action="store_true", help="also compare with the reference aligner's SAM")
    ap.add_argument("--nchrom", type=int, default=8)
    ap.add_argument("--gseed", type=int, default=2024)
    ap.add_argument("--driver", default=os.path.join(ROOT, "tests", "cpp", "test_e2e_oracle"))
    args, extra = ap.parse_known_args()
    import numpy as np
    import simdata as sd
    import bench
    from bt2x import lib

    wd = "/tmp/bt2x_hostprof"
    os.makedirs(wd, exist_ok=True)
    tag = f"g{int(args.mb * 1e6)}" + (f"_c{args.nchrom}" if args.nchrom != 8 else "")
    base = os.path.join(wd, tag)
    chroms = sd.gen_genome(int(args.mb * 1e6), nchrom=args.nchrom, seed=args.gseed)
    if not os.path.exists(base + ".4.bt2l"):
        fa = base + ".fa"
        sd.write_fasta(fa, chroms)
        t0 = time.time()
        lib.build_index(fa, base)
        print(f"# index {tag} built in {time.time() - t0:.1f} s", file=sys.stderr)
    fq = os.path.join(wd, f"{tag}_r{args.reads}_L{args.read_len}.fq")
    if not os.path.exists(fq):
        genome, starts = sd.concat_genome(chroms)
        reads, quals = sd.sim_reads_fast(genome, starts, args.reads, args.read_len, seed=3)
        sd.write_fastq_fixed(fq, reads, quals)
    sam = os.path.join(wd, "out.sam")
    cmd = [args.driver, base, fq, "--host-timing", "-p", str(args.p),
           "--slots", str(args.slots), "--dpad", str(args.dpad)] + extra
    t0 = time.time()
    with open(sam, "wb") as f:
        r = subprocess.run(cmd, stdout=f, stderr=subprocess.PIPE, text=True)
    print("\n".join(ln for ln in r.stderr.splitlines() if "HOST_TIMING" in ln or "PHASE" in ln or "error" in ln.lower())[-6000:], file=sys.stderr)
    print(f"# total {time.time() - t0:.1f} s", file=sys.stderr)
    if r.returncode:
        raise SystemExit(r.returncode)
    if args.check:
        ref = os.path.join(ROOT, "oracle", "_ref", "bowtie2-align-l")
        rsam = os.path.join(wd, "ref.sam")
        env = dict(os.environ, OMP_NUM_THREADS=str(args.p))
        subprocess.run([ref, "-x", base, "-U", fq, "-S", rsam, "--dpad", str(args.dpad)], env=env, check=True,
                       capture_output=True)
        a = bench.sam_records(sam)
        b = bench.sam_records(rsam)
        diff = sum(1 for x, y in zip(a, b) if x != y) + abs(len(a) - len(b))
        print(f"# parity vs reference: {diff} of {len(b)} records differ", file=sys.stderr)


if __name__ == "__main__":
    main()
