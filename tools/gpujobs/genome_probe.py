"""Probe: time the C3-scale synthetic genome + index build on the box."""
import os, sys, time
sys.path.insert(0, "tools"); sys.path.insert(0, "omp-bowtie2-prime_amd")
import numpy as np
import simdata as sd
t0 = time.time()
def mark(m):
    print(f"{time.time() - t0:8.1f}s {m}", flush=True)
total = int(float(sys.argv[1]) * 1e6)
chroms = sd.gen_genome(total, nchrom=24, seed=2024)
mark(f"genome {total}")
wd = "/tmp/probe"; os.makedirs(wd, exist_ok=True)
fa = wd + "/g.fa"
sd.write_fasta(fa, chroms)
mark("fasta written")
codes, starts = sd.concat_genome(chroms)
mark("concat")
import torch
import gpu_sa
x = codes[codes < 4]
mark(f"joined {len(x)}")
sa, bwt, keys = gpu_sa.suffix_array(x, device="cuda")
mark("gpu sa")
from bt2x import lib
lib.build_index_sa(fa, wd + "/g", sa, bwt=bwt, keys=keys)
mark("index files")
del sa, bwt, keys
idx = lib.Index(wd + "/g", load_offs=True)
mark("index loaded")
ctx = lib.Context(idx)
mark("context open (blocks + full SA in HBM)")
os.system(f"ls -la {wd}; free -g | head -2")
