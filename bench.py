#!/usr/bin/env python3
"""bench.py — BASELINE.json's headline metric on MI355X: 150 bp single-end reads,
end-to-end alignment with --dpad 12 (config C3; hg38 is not available offline, so a
seeded 1 Gbp synthetic genome stands in), reads/s and the DP kernel's HBM roofline.

Per rank (one process per GPU):
  1. The aligner itself, bt2x-align (FASTQ -> SAM; host driver + the three gfx950
     kernels, omp-bowtie2-prime_amd/host), runs once over the batch of --reads reads and
     records the inputs of every GPU launch it makes (--dump): the seed searches, SA
     resolutions and DP rounds that SwDriver::extendSeeds generates for these reads.
     A second, undumped run gives the end-to-end wall time (`end_to_end`, FASTQ parse,
     host logic, PCIe and SAM formatting included).
  2. The timed hot path: one step = that exact launch sequence replayed from HBM
     (inputs resident before the timed region) -- seed_kernel, resolve_kernel and
     dp_fill_kernel launches in the aligner's order.
     value = reads of all ranks / max-over-ranks wall time of K steps.
  3. Rank 0 at N=1: the reference aligner (oracle/_ref/bowtie2-align-l, OpenMP) on a
     bounded sample of the same FASTQ = cpu_baseline; its SAM is compared with ours
     record by record (`parity`).
Multi-GPU: reads sharded (each rank its own seeded batch), index replicated per GPU,
no collective on the data path ("scaling": "weak"); the only collective is the
max-of-times reduction for the report.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "omp-bowtie2-prime_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured copy
ALIGN = os.path.join(ROOT, "omp-bowtie2-prime_amd", "bt2x", "bt2x-align")
REF_ALIGN = os.path.join(ROOT, "oracle", "_ref", "bowtie2-align-l")


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
    ap.add_argument("--host-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")),
                    help="host threads of bt2x-align (the box's CPU share)")
    ap.add_argument("--cpu-sample", type=int, default=200000,
                    help="reads aligned by the reference aligner for cpu_baseline / parity")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")),
                    help="OpenMP threads of the reference CPU baseline (the box's CPU share)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--replay-ablate", type=int, default=0,
                    help="profiling only: BT2X_DP_ABLATE for the replay (1: DP fill without the walk); outputs invalid")
    ap.add_argument("--prep-only", action="store_true",
                    help="write the genome index and reads, print their paths, exit (profiling the aligner)")
    ap.add_argument("--lookahead", type=int, default=8, help="bt2x-align --lookahead (DP problems posed per request)")
    ap.add_argument("--slots", type=int, default=1 << 17,
                    help="bt2x-align --slots (reads in flight) of the end-to-end run; the launch-recording run "
                         "batches the whole --reads batch (--slots = --reads, --no-pipeline)")
    ap.add_argument("--rss-limit-gb", type=float, default=120.0, help="kill bt2x-align above this host RSS")
    return ap.parse_args()


def workload_key(args) -> str:
    g = f"synthetic{args.genome_mb:g}Mbp_s{args.genome_seed}" if args.genome == "synthetic" else args.genome
    return f"e2e|{g}|reads{args.reads}|R{args.read_len}|dpad{args.dpad}|la{args.lookahead}|round"


def pmc_traffic(args, kernel: str):
    """Per-step HBM bytes of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/<tag>_traffic.json, tools/pmc_traffic.py) taken on this same workload;
    (None, None) if there is none."""
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


def mark(msg):
    rss = 0
    try:
        with open("/proc/self/status") as f:
            rss = next(int(ln.split()[1]) >> 10 for ln in f if ln.startswith("VmRSS"))
    except (OSError, StopIteration):
        pass
    print(f"# {msg} (bench RSS {rss} MiB)", file=sys.stderr, flush=True)


def write_fastq(path, reads, quals, first_id=0):
    """Fixed-length FASTQ, vectorised: '@r<9 digits>' names."""
    n, R = reads.shape
    rec = np.empty((n, 11 + 1 + R + 3 + R + 1), dtype=np.uint8)
    rec[:, 0] = ord("@"); rec[:, 1] = ord("r")
    ids = np.arange(first_id, first_id + n, dtype=np.int64)
    for k in range(9):
        rec[:, 10 - k] = ord("0") + (ids // (10 ** k)) % 10
    rec[:, 11] = ord("\n")
    rec[:, 12:12 + R] = np.frombuffer(b"ACGTN", np.uint8)[reads]
    rec[:, 12 + R] = ord("\n"); rec[:, 13 + R] = ord("+"); rec[:, 14 + R] = ord("\n")
    rec[:, 15 + R:15 + 2 * R] = quals
    rec[:, 15 + 2 * R] = ord("\n")
    with open(path, "wb") as f:
        f.write(rec.tobytes())


def run_aligner(args, base, fq, sam, gpu, dump=None):
    """dump: record the launch sequence with the whole batch in flight (the largest
    launches; the problems are the same at any batching); otherwise the end-to-end
    configuration (--slots reads in flight, GPU launches overlapped with host work)."""
    slots = args.reads if dump else args.slots
    cmd = [ALIGN, "-x", base, "-U", fq, "-S", sam, "--dpad", str(args.dpad), "--device", str(gpu),
           "-p", str(args.host_threads), "--slots", str(slots), "--lookahead", str(args.lookahead), "--stats"]
    if dump:
        cmd += ["--dump", dump, "--no-pipeline"]
    t0 = time.perf_counter()
    errp = os.path.join(os.path.dirname(sam), "align.err")
    with open(errp, "w") as ferr:
        p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=ferr)
        peak = 0
        while p.poll() is None:          # host-RAM watchdog (the box caps a command's RAM)
            try:
                with open(f"/proc/{p.pid}/status") as f:
                    for ln in f:
                        if ln.startswith("VmRSS"):
                            peak = max(peak, int(ln.split()[1]) >> 10)
            except OSError:
                pass
            if peak > args.rss_limit_gb * 1024 or time.perf_counter() - t0 > 1500:
                p.kill()
                p.wait()
                break
            time.sleep(0.2)
    wall = time.perf_counter() - t0
    err = open(errp).read()
    if p.returncode != 0:
        raise SystemExit(f"bt2x-align failed (rc {p.returncode}, peak RSS {peak} MiB): {err[-3000:]}")
    print(f"# bt2x-align {'(dump) ' if dump else ''}{wall:.1f} s, peak RSS {peak} MiB", file=sys.stderr, flush=True)
    line = [ln for ln in err.splitlines() if ln.startswith("BT2X_STATS")][-1]
    st = {k: float(v) for k, v in (t.split("=") for t in line.split()[1:])}
    ru = [ln for ln in err.splitlines() if ln.startswith("BT2X_RUSAGE_ALIGN")]
    if ru:
        st["rusage_align"] = {k: float(v) for k, v in (t.split("=") for t in ru[-1].split()[1:])}
    gl = [ln for ln in err.splitlines() if ln.startswith("BT2X_GPU")]
    if gl:
        st["gpu"] = {k: float(v) for k, v in (t.split("=") for t in gl[-1].split()[1:])}
    st["wall_incl_index_load"] = wall
    st["peak_rss_mib"] = peak
    st["summary"] = [ln.strip() for ln in err.splitlines() if "aligned" in ln or "overall" in ln]
    return st


def load_dumps(ddir):
    """-> list of (kind, [arrays]) in launch order (DumpBackend, bt2x_align_main.cpp)."""
    from bt2x import abi
    out = []
    for path in sorted(glob.glob(os.path.join(ddir, "*.*"))):
        kind = path.rsplit(".", 1)[1]
        nparts = {"seed": 2, "resolve": 1, "dp": 5, "round": 5}[kind]
        raw = np.fromfile(path, dtype=np.uint8)
        sizes = raw[:8 * nparts].view(np.uint64).astype(np.int64)
        parts, o = [], 8 * nparts
        for s in sizes:
            parts.append(raw[o:o + s]); o += s
        if kind == "seed":
            parts[1] = parts[1].view(abi.SEED_IN)
        elif kind == "resolve":
            parts[0] = parts[0].view(abi.RESOLVE_IN)
        elif kind == "round":
            parts[1] = parts[1].view(abi.SEED_IN)
            parts[2] = parts[2].view(abi.ROUND_IN)
            parts[3] = parts[3].view(abi.EXRANGE)
            parts[4] = parts[4].view(np.uint64)
        else:
            parts[3] = parts[3].view(abi.DP_IN)
            parts[4] = parts[4].view(np.uint64)
        out.append((kind, parts))
    return out


def sam_records(path, limit_ids=None):
    recs = []
    with open(path, "rb") as f:
        for ln in f:
            if ln.startswith(b"@"):
                continue
            if limit_ids is not None and int(ln[1:10]) >= limit_ids:
                continue
            recs.append(ln.rstrip(b"\n"))
    recs.sort()
    return recs


def cpu_reference(args, base, fq_sample, m, workdir):
    """The reference aligner (OpenMP, --cpu-threads) on the first m reads; alignment time
    = wall(m reads) - wall(1 read) (index load cancels)."""
    if not os.access(REF_ALIGN, os.X_OK):
        return None, None
    env = dict(os.environ, OMP_NUM_THREADS=str(args.cpu_threads), OMP_WAIT_POLICY="ACTIVE")
    one = os.path.join(workdir, "one.fq")
    with open(fq_sample, "rb") as f, open(one, "wb") as g:
        for _ in range(4):
            g.write(f.readline())
    times = []
    for fq, sam in ((one, os.path.join(workdir, "ref_one.sam")), (fq_sample, os.path.join(workdir, "ref.sam"))):
        t0 = time.perf_counter()
        r = subprocess.run([REF_ALIGN, "-x", base, "-U", fq, "-S", sam, "--dpad", str(args.dpad)],
                           env=env, capture_output=True, text=True, timeout=1200)
        times.append(time.perf_counter() - t0)
        if r.returncode != 0:
            print(r.stderr[-2000:], file=sys.stderr)
            return None, None
    dt = max(times[1] - times[0], 1e-6)
    base_line = {"value": round(m / dt / 1e6, 6), "unit": "M reads/s", "cores": args.cpu_threads,
                 "kind": "reference",
                 "sample": f"first {m} reads of this batch through the reference aligner "
                           f"(oracle/_ref/bowtie2-align-l --dpad {args.dpad}, FASTQ->SAM, OpenMP "
                           f"{args.cpu_threads} threads): {times[1]:.2f} s minus {times[0]:.2f} s index load"}
    return base_line, os.path.join(workdir, "ref.sam")


def main():
    args = parse()
    import torch
    from bt2x import dist as bdist
    rank, world, local = bdist.world()
    # rehearsal knobs (not used by the driver): BT2X_BENCH_DEVICE pins every rank to one
    # GPU, BT2X_BENCH_DIST_BACKEND=gloo runs the rank reductions on the host
    gpu = int(os.environ.get("BT2X_BENCH_DEVICE", local))
    backend = os.environ.get("BT2X_BENCH_DIST_BACKEND", "nccl")
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            torch.cuda.set_device(gpu)
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)

    from bt2x import abi, lib
    import simdata as sd

    workdir = os.path.join("/tmp", f"bt2x_bench_{os.getuid()}")
    os.makedirs(workdir, exist_ok=True)
    chroms, base, gdesc = load_genome(args, workdir, rank, dist)
    genome, starts = sd.concat_genome(chroms)
    R, n = args.read_len, args.reads
    reads, quals, _, _, _ = sd.sim_reads_fixed(genome, starts, n, R, seed=bdist.rank_seed(3, rank))
    del genome
    rdir = os.path.join(workdir, f"rank{rank}")
    os.makedirs(rdir, exist_ok=True)
    fq = os.path.join(rdir, "reads.fq")
    write_fastq(fq, reads, quals)
    del reads, quals
    mark(f"{n} reads written to {fq}")
    if args.prep_only:
        print(f"BT2X_DATA {base} {fq}", flush=True)
        return

    # ---- 1. the aligner: launch recording run, then the end-to-end timing run
    ddir = os.path.join(rdir, "dump")
    for p in glob.glob(os.path.join(ddir, "*")):
        os.unlink(p)
    os.makedirs(ddir, exist_ok=True)
    sam = os.path.join(rdir, "out.sam")
    run_aligner(args, base, fq, sam, gpu, dump=ddir)
    e2e = run_aligner(args, base, fq, sam, gpu)
    launches = load_dumps(ddir)
    mark(f"{len(launches)} launches loaded")

    # ---- 2. replay the launch sequence from HBM
    if args.replay_ablate:
        os.environ["BT2X_DP_ABLATE"] = str(args.replay_ablate)
    if world == 1 or backend != "nccl":
        torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    idx = lib.Index(base, load_offs=True)     # SA sample + text: full SA rebuilt in HBM
    ctx = lib.Context(idx, device=gpu)

    def to_dev(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)

    plan = []
    for kind, parts in launches:
        if kind == "seed":
            m = len(parts[1])
            plan.append((kind, m, [to_dev(parts[0]), to_dev(parts[1]),
                                   torch.empty(m * abi.SEED_OUT.itemsize, dtype=torch.uint8, device=dev)]))
        elif kind == "resolve":
            m = len(parts[0])
            plan.append((kind, m, [to_dev(parts[0]),
                                   torch.empty(m * abi.RESOLVE_OUT.itemsize, dtype=torch.uint8, device=dev)]))
        elif kind == "round":
            m = len(parts[2])
            meta = parts[4]
            caps = [int(meta[1]) + 1024, int(meta[2]) + 1024, int(meta[3]) + 256]   # sizes the aligner saw
            exr = parts[3] if len(parts[3]) else np.zeros(1, dtype=abi.EXRANGE)
            plan.append((kind, m, [to_dev(parts[0]), to_dev(parts[1]), len(parts[1]), to_dev(parts[2]), to_dev(exr),
                                   int(meta[0]),
                                   torch.empty(m * abi.ROUND_OUT.itemsize, dtype=torch.uint8, device=dev),
                                   torch.empty(caps[0] * abi.SAT.itemsize, dtype=torch.uint8, device=dev), caps[0],
                                   torch.empty(caps[1] * abi.RESOLVE_OUT.itemsize, dtype=torch.uint8, device=dev), caps[1],
                                   torch.empty(caps[2] * abi.EXRANGE.itemsize, dtype=torch.uint8, device=dev), caps[2],
                                   torch.zeros(4, dtype=torch.int32, device=dev)]))
        else:
            m = len(parts[3])
            rec_cap, edit_cap = int(parts[4][0]) + 1024, int(parts[4][1]) + 4096   # sizes the aligner saw
            plan.append((kind, m, [to_dev(parts[0]), to_dev(parts[1]), to_dev(parts[2]), to_dev(parts[3]),
                                   torch.empty(m * abi.DP_OUT.itemsize, dtype=torch.uint8, device=dev),
                                   torch.empty(rec_cap * abi.ALN_REC.itemsize, dtype=torch.uint8, device=dev),
                                   torch.empty(edit_cap * 4, dtype=torch.uint8, device=dev),
                                   torch.zeros(16, dtype=torch.int32, device=dev), rec_cap, edit_cap]))
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    kid = {"seed": abi.K_SEED, "resolve": abi.K_RESOLVE, "dp": abi.K_DP, "round": abi.K_ROUND}
    units = {"seed": 0, "resolve": 0, "dp": 0, "round": 0}
    for kind, m, b in plan:
        units[kind] += m
        if kind == "round":
            units["seed"] += b[2]

    def step(record=None, counters=None):
        for kind, m, b in plan:
            if kind == "seed":
                ctx.seed_search_dev(b[0].data_ptr(), b[1].data_ptr(), m, b[2].data_ptr(), True, sh)
            elif kind == "resolve":
                ctx.resolve_dev(b[0].data_ptr(), m, b[1].data_ptr(), False, sh)
            elif kind == "round":
                ctx.seed_round_dev(b[0].data_ptr(), b[1].data_ptr(), b[2], b[3].data_ptr(), m, b[4].data_ptr(), b[5],
                                   b[6].data_ptr(), b[7].data_ptr(), b[8], b[9].data_ptr(), b[10], b[11].data_ptr(),
                                   b[12], b[13].data_ptr(), sh)
            else:
                ctx.dp_align_dev(b[0].data_ptr(), b[1].data_ptr(), b[2].data_ptr(), b[3].data_ptr(), m,
                                 b[4].data_ptr(), b[5].data_ptr(), b[8], b[6].data_ptr(), b[9],
                                 b[7].data_ptr(), sh)
            if record is not None:
                # HIP events recorded on this stream around each launch (bt2x_last_kernel_ms);
                # a round's seed kernel and ranking+resolution are also booked as seed / resolve
                record[kind]["ms"] += ctx.last_kernel_ms(kid[kind])
                if kind == "round":
                    record["seed"]["ms"] += ctx.last_kernel_ms(abi.K_SEED)
                    record["resolve"]["ms"] += ctx.last_kernel_ms(abi.K_RESOLVE)
            if counters is not None:
                for kk in (("seed", "resolve") if kind == "round" else (kind,)):
                    for k, v in ctx.last_counters(kid[kk]).items():
                        counters[kk][k] = counters[kk].get(k, 0) + v
                if kind == "round":
                    rs = ctx.last_round_stats()
                    for k in ("reads", "jobs", "samples"):
                        counters["round"][k] = counters["round"].get(k, 0) + rs[k]
                    counters["round"]["max_samples"] = max(counters["round"].get("max_samples", 0), rs["max_samples"])

    ctr = {k: {} for k in kid}          # algorithmic-work counters (deterministic per step)
    for w in range(max(args.warmup, 1)):
        step(counters=ctr if w == 0 else None)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    recs = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rec = {k: {"ms": 0.0} for k in kid}
        step(rec)
        recs.append(rec)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    e2e_t = e2e["t_align"]
    if dist:
        dist.barrier()
        red_dev = dev if backend == "nccl" else None
        elapsed = bdist.max_over_ranks(elapsed, dist, red_dev)
        e2e_t = bdist.max_over_ranks(e2e_t, dist, red_dev)
    for kind, m, b in plan:           # overflow check on the last step's arenas
        if kind == "dp":
            used = b[7][:2].cpu().numpy()
            if used[0] > b[8] or used[1] > b[9]:
                raise SystemExit(f"DP result arena overflow {used} vs {(b[8], b[9])}")

    value = n * world * args.steps / elapsed / 1e6
    kms = {k: float(np.mean([r[k]["ms"] for r in recs])) for k in kid}
    # algorithmic bytes: FM = 128*(2*BiLF + LF1) + 16*ftab (+ 128*LF1 + 8 per
    # SA sample for the GroupWalk resolve); DP = 3*R*C (E,F,H) + C (window) + 10*ceil(R/16)*16
    cs, cr, cd = ctr["seed"], ctr["resolve"], ctr["dp"]
    fm_bytes = 128 * (2 * cs.get("n_bilf", 0) + cs.get("n_lf1", 0)) + 16 * cs.get("n_ftab", 0)
    res_bytes = cr.get("alg_bytes", 0)
    dp_bytes = 3 * cd.get("dp_cells", 0) + cd.get("dp_cols", 0) + units["dp"] * 10 * ((R + 15) // 16) * 16
    kern = {"seed": (kms["seed"], fm_bytes), "resolve": (kms["resolve"], res_bytes), "dp": (kms["dp"], dp_bytes)}
    # (round launches are booked above as their seed and resolve parts)
    dom = max(kern, key=lambda k: kern[k][0])
    ach = kern[dom][1] / (kern[dom][0] / 1e3) / 1e9 if kern[dom][0] > 0 else 0.0
    traffic, traffic_src = pmc_traffic(args, dom)
    # the kernel's own algorithmic bytes (bt2x_counters.alg_bytes: for the DP, the 1 B
    # traceback flag per cell it writes + window + read/quality bytes), beside §8(d)'s
    # reference-equivalent figure above
    own = {"seed": cs.get("alg_bytes", 0), "resolve": cr.get("alg_bytes", 0), "dp": cd.get("alg_bytes", 0)}[dom]
    ach_own = own / (kern[dom][0] / 1e3) / 1e9 if kern[dom][0] > 0 else 0.0
    nl = {k: sum(1 for kk, _, _ in plan if kk == k) for k in kid}
    nl["seed"] += nl["round"]
    nl["resolve"] += nl["round"]
    line = {
        "metric": "M reads/s aligned (150 bp SE vs hg38) at 1/2/4/8 MI355X; % HBM-roofline",
        "value": round(value, 4), "unit": "M reads/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded genome + simulated 150 bp reads, BASELINE.md error model)",
        "config": {"workload": f"C3 stand-in: {R} bp SE, --dpad {args.dpad}, genome {gdesc}; step = the "
                               f"GPU launch sequence bt2x-align issues to align {n} reads end to end "
                               f"({nl['round']} seed-round launches (seed search + ranking/prioritization + SA "
                               f"resolution), {nl['seed'] - nl['round']} seed, {nl['resolve'] - nl['round']} resolve, "
                               f"{nl['dp']} DP launches: {units['seed']} seeds, {cr.get('n_problems', 0)} SA "
                               f"elements, {units['dp']} DP problems), replayed from HBM",
                   "reads_per_gpu_step": n, "read_len": R, "parallelism": f"dp{world} (read shards)",
                   "key": workload_key(args)},
        # achieved = algorithmic bytes per launch / average launch time (= per-step bytes / per-step
        # kernel time); traffic (PMC, committed per step) is reported per launch to match.
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                     "traffic": None if traffic is None else int(traffic / max(nl[dom], 1)),
                     "alg_bytes": int(kern[dom][1] / max(nl[dom], 1)),
                     "avg_launch_ms": round(kern[dom][0] / max(nl[dom], 1), 4), "per": "launch",
                     "alg_bytes_per_step": kern[dom][1], "traffic_per_step": traffic,
                     "launches_per_step": nl[dom], "traffic_src": traffic_src,
                     "alg_bytes_note": "achieved/alg_bytes count SURVEY 8(d)'s reference-equivalent bytes (3 B of "
                                       "E/F/H per DP cell); the kernel itself moves 1 B per cell: see achieved_kernel",
                     "achieved_kernel": round(ach_own, 2), "frac_kernel": round(ach_own / HBM_PEAK_GBS, 4),
                     "alg_bytes_kernel": int(own / max(nl[dom], 1))},
        "kernels": {"seed_ms": round(kms["seed"], 3), "resolve_ms": round(kms["resolve"], 3),
                    "dp_ms": round(kms["dp"], 3), "seed_alg_bytes": fm_bytes, "resolve_alg_bytes": res_bytes,
                    "dp_alg_bytes": dp_bytes, "launches": nl, "units": units,
                    "counters_seed": cs, "counters_resolve": cr, "counters_dp": cd,
                    "round_sampling": ctr["round"]},
        "end_to_end": {"value": round(n * world / e2e_t / 1e6, 4), "unit": "M reads/s",
                       "what": "bt2x-align FASTQ->SAM wall time (host driver, PCIe, SAM formatting; "
                               f"index load excluded; --slots {args.slots}, launches overlapped with host "
                               "work), max over ranks",
                       "t_align_s": round(e2e_t, 3), "summary": e2e["summary"],
                       "stats": {k: v for k, v in e2e.items() if k not in ("summary",)}},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        m = min(args.cpu_sample, n)
        fqs = os.path.join(rdir, "sample.fq")
        with open(fq, "rb") as f, open(fqs, "wb") as g:
            rec_len = 11 + 1 + R + 3 + R + 1
            g.write(f.read(rec_len * m))
        ref, ref_sam = cpu_reference(args, base, fqs, m, rdir)
        if ref is not None:
            line["cpu_baseline"] = ref
            ours, theirs = sam_records(sam, limit_ids=m), sam_records(ref_sam)
            diff = sum(1 for a, b in zip(ours, theirs) if a != b) + abs(len(ours) - len(theirs))
            line["parity"] = {"sample_reads": m, "records_differ": diff,
                              "what": "sorted SAM records of bt2x-align vs the reference aligner on the sample"}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
