#!/usr/bin/env python3
"""bench.py — throughput of the MI355X hot path (FM seed search + banded end-to-end DP)
on BASELINE.json's headline workload: 150 bp single-end reads, u8 DP with --dpad 12
(config C3; hg38 is not available offline, so a seeded synthetic genome stands in).

One step = the hot path over one batch of synthetic reads already resident in HBM:
  1. bt2x_seed_search_dev: exact search + left extension of every instantiated seed
     (18 seeds/read at 150 bp: 9 per strand, MultiSeedAligner::searchAllSeedsDoAll);
  2. bt2x_dp_align_dev: one framed end-to-end DP problem per read at its seed-hit
     diagonal (SwAligner::align + every nextAlignment() call), exactly as
     SwDriver::extendSeeds frames it (the reference measures 1.04 DP/read).
value = reads of all ranks / max-over-ranks wall time of K steps (M reads/s).

Multi-GPU: one process per GPU, reads sharded (each rank its own seeded batch), index
replicated per GPU, no collective on the data path ("scaling": "weak"); the only
collective is the max-of-times reduction for the report.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "omp-bowtie2-prime_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured copy


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--reads", type=int, default=1 << 20, help="reads per step per GPU")
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--dpad", type=int, default=12, help="--dpad (maxhalf); 12 fits 150 bp in ALN_MAX_COLS")
    ap.add_argument("--genome", default="synthetic", help="'synthetic' (default) or 'rep' (fixture)")
    ap.add_argument("--genome-mb", type=float, default=1000.0)
    ap.add_argument("--genome-seed", type=int, default=2024)
    ap.add_argument("--cpu-sample", type=int, default=200000,
                    help="reads timed on the reference's CPU path (oracle/_ref/refharness bench)")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")),
                    help="OpenMP threads for the reference CPU baseline (the box's CPU share)")
    ap.add_argument("--port-sample", type=int, default=20000, help="reads timed on the 1-thread C port")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--overlap", type=int, default=0, help="1: seed and DP stages on two streams")
    return ap.parse_args()


def workload_key(args) -> str:
    g = f"synthetic{args.genome_mb:g}Mbp_s{args.genome_seed}" if args.genome == "synthetic" else args.genome
    return f"{g}|reads{args.reads}|R{args.read_len}|dpad{args.dpad}"


def pmc_traffic(args, kernel: str):
    """Per-launch HBM bytes of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/<tag>_traffic.json, tools/pmc_traffic.py) taken on this same workload;
    (None, None) if there is none."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), reverse=True):
        with open(path) as f:
            t = json.load(f)
        if t.get("workload") == workload_key(args) and kernel in t.get("kernels", {}):
            return t["kernels"][kernel]["traffic_bytes"], os.path.relpath(path, ROOT)
    return None, None


def load_genome(args, workdir, rank=0, dist=None):
    """-> (chroms, index basename, description).  'synthetic' (default): a seeded
    genome-scale reference (tools/simdata.gen_genome: 24 chromosomes, interspersed
    repeat families, low-complexity stretches, N runs) indexed here -- suffix array
    by prefix doubling on the GPU (tools/gpu_sa.py), files by bt2x_build_index_sa
    (byte-identical to the reference's bowtie2-build-l, tests/test_builder.py).
    Index building is setup, outside the timed region."""
    import golden_io as g
    import simdata as sd
    if args.genome == "rep":
        import lzma
        with lzma.open(os.path.join(g.GOLDEN, "rep.fa.xz"), "rb") as f:
            raw = f.read()
        path = os.path.join(workdir, f"rep{rank}.fa")
        with open(path, "wb") as f:
            f.write(raw)
        chroms = sd.read_fasta(path)
        base = g.materialize_index("rep", os.path.join(workdir, f"r{rank}"))
        return chroms, base, "rep (300 kbp repeat-rich fixture)"
    if args.genome != "synthetic":
        raise SystemExit("--genome must be 'synthetic' or 'rep'")
    import gpu_sa
    from bt2x import lib
    total = int(args.genome_mb * 1e6)
    tag = f"syn{total}_s{args.genome_seed}"
    base = os.path.join(workdir, tag)
    fa = base + ".fa"
    t0 = time.perf_counter()
    chroms = sd.gen_genome(total, nchrom=24, seed=args.genome_seed)
    # rank 0 builds (ranks share the node's /tmp); the others wait at the barrier
    if rank == 0 and not all(os.path.exists(f"{base}.{k}.bt2l") for k in "1234"):
        sd.write_fasta(fa, chroms)
        codes, _ = sd.concat_genome(chroms)
        sa, bwt, keys = gpu_sa.suffix_array(codes[codes < 4], device="cuda")
        lib.build_index_sa(fa, base + ".tmp", sa, bwt=bwt, keys=keys)
        for k in "1234":
            os.replace(f"{base}.tmp.{k}.bt2l", f"{base}.{k}.bt2l")
        del sa, bwt, keys, codes
        os.unlink(fa)
        import torch
        torch.cuda.empty_cache()
    if dist:
        dist.barrier()
    print(f"# genome {tag}: {total / 1e6:.0f} Mbp, index ready in {time.perf_counter() - t0:.1f} s",
          file=sys.stderr, flush=True)
    return chroms, base, f"synthetic {total / 1e6:.0f} Mbp (seed {args.genome_seed}, 24 chromosomes, " \
                         f"5% repeat families, low-complexity, N runs)"


def main():
    args = parse()
    import torch
    from bt2x import dist as bdist
    rank, world, local = bdist.world()
    # rehearsal knobs (not used by the driver): BT2X_BENCH_DEVICE pins every rank to one
    # GPU, BT2X_BENCH_DIST_BACKEND=gloo runs the rank reductions on the host
    gpu = int(os.environ.get("BT2X_BENCH_DEVICE", local))
    backend = os.environ.get("BT2X_BENCH_DIST_BACKEND", "nccl")
    torch.cuda.set_device(gpu)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)

    from bt2x import abi, framing, lib, seeds
    import simdata as sd

    workdir = os.path.join("/tmp", f"bt2x_bench_{os.getuid()}")
    os.makedirs(workdir, exist_ok=True)
    chroms, base, gdesc = load_genome(args, workdir, rank, dist)
    genome, starts = sd.concat_genome(chroms)
    lens = np.array([len(s) for _, s in chroms], dtype=np.int64)

    R = args.read_len
    n = args.reads
    reads, quals, chrom, off, fw = sd.sim_reads_fixed(genome, starts, n, R, seed=bdist.rank_seed(3, rank))
    # host prep (untimed): seeds and DP problems
    sbuf, sin, _ = seeds.batch_fixed_length(reads)
    drd, dqu, drf, dpin, keep = framing.build_dp_batch_fixed(genome, starts, lens, chrom, off, fw,
                                                             reads, quals, maxhalf=args.dpad)
    nseed, ndp = len(sin), len(dpin)

    idx = lib.Index(base, load_offs=True)     # SA sample + text: full SA rebuilt in HBM
    ctx = lib.Context(idx, device=gpu)
    dev = torch.device("cuda", gpu)

    def to_dev(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)

    d_sbuf, d_sin = to_dev(sbuf), to_dev(sin)
    d_sout = torch.empty(nseed * abi.SEED_OUT.itemsize, dtype=torch.uint8, device=dev)
    d_rd, d_qu, d_rf, d_dpin = to_dev(drd), to_dev(dqu), to_dev(drf), to_dev(dpin)
    d_dpout = torch.empty(ndp * abi.DP_OUT.itemsize, dtype=torch.uint8, device=dev)
    rec_cap, edit_cap = 4 * ndp + 1024, 48 * ndp + 4096
    d_recs = torch.empty(rec_cap * abi.ALN_REC.itemsize, dtype=torch.uint8, device=dev)
    d_edits = torch.empty(edit_cap * 4, dtype=torch.uint8, device=dev)
    d_cnt = torch.zeros(16, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    # --overlap: the seed stage and the DP stage on two HIP streams, the way a streaming
    # aligner pipelines seed(batch k+1) with DP(batch k); the seed kernel is latency-bound
    # and the DP fill VALU-bound, so they share the CUs well.  Every step still runs both
    # stages over the whole batch; the timed region waits for both streams.
    s2 = torch.cuda.Stream(dev) if args.overlap else stream
    sh2 = s2.cuda_stream

    def step():
        if args.overlap:
            s2.wait_stream(stream)
        ctx.seed_search_dev(d_sbuf.data_ptr(), d_sin.data_ptr(), nseed, d_sout.data_ptr(), True, sh2)
        ctx.dp_align_dev(d_rd.data_ptr(), d_qu.data_ptr(), d_rf.data_ptr(), d_dpin.data_ptr(), ndp,
                         d_dpout.data_ptr(), d_recs.data_ptr(), rec_cap, d_edits.data_ptr(),
                         edit_cap, d_cnt.data_ptr(), sh)
        if args.overlap:
            stream.wait_stream(s2)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    seed_ms, dp_ms = [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        # per-kernel durations from HIP events recorded on this stream around each launch
        seed_ms.append(ctx.last_kernel_ms(abi.K_SEED))
        dp_ms.append(ctx.last_kernel_ms(abi.K_DP))
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
        elapsed = bdist.max_over_ranks(elapsed, dist, dev if backend == "nccl" else None)
    used = d_cnt[:2].cpu().numpy()
    if used[0] > rec_cap or used[1] > edit_cap:
        raise SystemExit(f"result arena overflow {used} vs {(rec_cap, edit_cap)}")
    cs, cd = ctx.last_counters(abi.K_SEED), ctx.last_counters(abi.K_DP)

    # sanity: outputs of the last step
    sout = d_sout.cpu().numpy().view(abi.SEED_OUT)
    dout = d_dpout.cpu().numpy().view(abi.DP_OUT)
    aligned_frac = float((dout["status"] == 1).mean())

    value = n * world * args.steps / elapsed / 1e6
    seed_avg, dp_avg = float(np.mean(seed_ms)), float(np.mean(dp_ms))
    # algorithmic bytes: FM = 128*(2*BiLF + LF1) + 16*ftab;
    # DP = 3*R*C (E,F,H) + C (window) + 10*ceil(R/16)*16 (profile) per problem
    fm_bytes = 128 * (2 * cs["n_bilf"] + cs["n_lf1"]) + 16 * cs["n_ftab"]
    dp_bytes = 3 * cd["dp_cells"] + cd["dp_cols"] + ndp * 10 * ((R + 15) // 16) * 16
    kern = {"seed": (seed_avg, fm_bytes), "dp": (dp_avg, dp_bytes)}
    dom = max(kern, key=lambda k: kern[k][0])
    ach = kern[dom][1] / (kern[dom][0] / 1e3) / 1e9
    traffic, traffic_src = pmc_traffic(args, dom)
    line = {
        "metric": "M reads/s aligned (150 bp SE vs hg38) at 1/2/4/8 MI355X; % HBM-roofline",
        "value": round(value, 4), "unit": "M reads/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded genome + simulated 150 bp reads, BASELINE.md error model)",
        "config": {"workload": f"C3 stand-in: {R} bp SE, --dpad {args.dpad}, genome {gdesc}; "
                               f"step = seed search+extend ({nseed} seeds) + DP ({ndp} problems)"
                               + (", the two stages on two streams" if args.overlap else ""),
                   "reads_per_gpu_step": n, "read_len": R, "parallelism": f"dp{world} (read shards)",
                   "key": workload_key(args)},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "alg_bytes": kern[dom][1], "traffic_src": traffic_src},
        "kernels": {"seed_ms": round(seed_avg, 3), "dp_ms": round(dp_avg, 3),
                    "seed_alg_bytes": fm_bytes, "dp_alg_bytes": dp_bytes,
                    "dp_traceback_bytes": cd["dp_cells"], "counters_seed": cs, "counters_dp": cd},
        "checks": {"dp_aligned_frac": round(aligned_frac, 4),
                   "seed_reported_frac": round(float(sout["need_reporting"].mean()), 4)},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        ref = cpu_baseline_reference(args, reads, quals, chrom, off, fw, base, workdir)
        port = cpu_baseline_port(args, sbuf, sin, drd, dqu, drf, dpin, base, n)
        line["cpu_baseline"] = ref if ref is not None else port
        if ref is not None:
            line["cpu_port"] = port
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


def cpu_baseline_reference(args, reads, quals, chrom, off, fw, base, workdir):
    """The reference's own seed search + DP (oracle/_ref/refharness bench: its
    MultiSeedAligner::searchAllSeedsDoAll and SwAligner::align/nextAlignment, OpenMP
    over --cpu-threads host cores) on the first --cpu-sample reads of this batch.
    None when the reference build did not travel with the snapshot."""
    import subprocess
    exe = os.path.join(ROOT, "oracle", "_ref", "refharness")
    if not os.access(exe, os.X_OK):
        return None
    m = min(args.cpu_sample, len(reads))
    fq = os.path.join(workdir, "cpu_sample.fq")
    alpha = np.frombuffer(b"ACGTN", dtype=np.uint8)
    with open(fq, "wb") as f:
        seqs, qs = alpha[reads[:m]], quals[:m]
        for i in range(m):
            f.write(b"@r%d:%d:%d:%d\n%s\n+\n%s\n" % (i, chrom[i], off[i], int(fw[i]),
                                                        seqs[i].tobytes(), qs[i].tobytes()))
    env = dict(os.environ, OMP_NUM_THREADS=str(args.cpu_threads), OMP_WAIT_POLICY="ACTIVE")
    out = subprocess.run([exe, "bench", base, fq, "--dpad", str(args.dpad)], env=env,
                         capture_output=True, text=True, timeout=900)
    if out.returncode != 0:
        print(out.stderr[-2000:], file=sys.stderr)
        return None
    kv = dict(t.split("=") for t in out.stdout.split("BENCH", 1)[1].split())
    dt = float(kv["seed_s"]) + float(kv["dp_s"])
    return {"value": round(m / dt / 1e6, 6), "unit": "M reads/s", "cores": int(kv["threads"]),
            "kind": "reference",
            "sample": f"{m} reads of this batch: {kv['seeds']} seeds searched+extended "
                      f"({float(kv['seed_s']):.2f} s) + {kv['dp_probs']} DP problems, "
                      f"{kv['dp_alns']} alignments ({float(kv['dp_s']):.2f} s); reference "
                      f"searchAllSeedsDoAll + SwAligner (oracle/_ref/refharness bench), "
                      f"OpenMP {kv['threads']} threads"}


def cpu_baseline_port(args, sbuf, sin, drd, dqu, drf, dpin, base, n):
    """The oracle ("port", 1 thread) on a bounded sample of the same workload."""
    import oracle_lib as ol
    m = min(args.port_sample, n)
    spr = len(sin) / n
    sseeds = sin[: int(round(spr * m))]
    sdp = dpin[: int(round(len(dpin) / n * m))]
    oidx = ol.OracleIndex(base)
    t0 = time.perf_counter()
    ol.seed_search(oidx, sbuf, sseeds, True)
    ol.dp_align(ol.default_scoring(), drd, dqu, drf, sdp, debug=False)
    dt = time.perf_counter() - t0
    return {"value": round(m / dt / 1e6, 6), "unit": "M reads/s", "cores": 1, "kind": "port",
            "sample": f"{m} reads: {len(sseeds)} seeds + {len(sdp)} DP problems, oracle/bt2x_oracle.c, "
                      f"{dt:.1f} s"}


if __name__ == "__main__":
    main()
