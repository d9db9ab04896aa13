#!/usr/bin/env python3
"""bench.py — BASELINE.json's headline metric on MI355X: end-to-end FASTQ -> SAM reads/s
of 150 bp single-end reads at --dpad 12 (config C3).  hg38 is not available offline: a
seeded 3.1 Gbp synthetic genome of 24 chromosomes stands in (tools/simdata.gen_genome:
interspersed repeat families, low-complexity stretches, N runs), indexed on the box.

Per rank (one process per GPU; the GPU work runs in bt2x-align, a child process):
  setup   genome (seeded, every rank), its index (rank 0: suffix array by prefix doubling
          on the GPU, tools/gpu_sa.py; files by bt2x_build_index_sa, byte-identical to the
          reference builder), and the rank's reads: W warmup + K step files of
          ceil(10M / K) reads each (tools/simdata.sim_reads_fast, BASELINE.md's error model),
          generated in a process pool before anything touches the GPU.
  timed   bt2x-align -U warm1,..,warmW,step1,..,stepK --warmup-files W: the W warmup files
          run untimed inside the same process (first launches, page faults, pools), then
          the K step files are one timed FASTQ -> SAM run: parse, the host driver, every
          seed search / SA resolution / DP on the GPU, PCIe, SAM formatting and writing.
          All ranks start it after a barrier; value = reads of all ranks / max over ranks
          of the timed run's wall time (BT2X_TIMED t_align; the index load is outside it).
  kernels rank 0: bt2x-align --dump records the GPU launches of one 1M-read file (a cohort
          of the timed run's size in flight, so the launches have its shapes); the
          launch sequence is replayed from HBM (inputs resident) with HIP events around
          each launch (bt2x_last_kernel_ms, on the launch stream) -> per-kernel time,
          the dominant kernel's roofline, and replay_reads_per_s (kernels alone).
  cpu     rank 0 at N=1: the reference aligner (oracle/_ref/bowtie2-align-l, OpenMP)
          on a bounded sample of the first step file (SURVEY §8(d) protocol: threads n-1
          and n of the box's CPU share, the better one repeated to a median of 3, plus a
          1-thread line; alignment time = wall - wall of a 1-read run (index load); the
          reference's own Timer: phase sums reported).  Its SAM is compared with ours
          record by record (`parity`).
Multi-GPU: each rank aligns its own 10M-read batch ("scaling": "weak"), the index
replicated per GPU; the ranks' only exchange is the final sum of the ReportingMetrics
counters and the max of the times (gloo: host values, no GPU collective on the path).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import shutil
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
C3_READS = 10_000_000


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10, help="timed step files (C3's 10M reads split K ways)")
    ap.add_argument("--warmup", type=int, default=1, help="untimed warmup files")
    ap.add_argument("--reads", type=int, default=C3_READS, help="timed reads per GPU (C3: 10M)")
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--dpad", type=int, default=12, help="--dpad (maxhalf); 12 fits 150 bp in ALN_MAX_COLS")
    ap.add_argument("--genome-mb", type=float, default=3100.0)
    ap.add_argument("--genome-seed", type=int, default=2024)
    ap.add_argument("--host-threads", type=int, default=0, help="bt2x-align -p (0: the rank's CPU share)")
    # (131,072: two cohorts of 65,536.  Round 6 measured 262,144 with malloc on huge pages: DP
    # launches twice as large put the DP at 0.387 of its roofline instead of 0.296 and C2's
    # i16 at 0.382, but the host-bound end-to-end rate fell 4.6 % over four interleaved pairs
    # and the repeat-heavy leg 14 %: profiles/r06s3_slots/, r06s4_slots/, r06b1_slots262144/)
    ap.add_argument("--slots", type=int, default=1 << 17, help="bt2x-align --slots (reads in flight)")
    ap.add_argument("--replay-reads", type=int, default=1 << 20, help="reads whose GPU launches are replayed")
    ap.add_argument("--replay-steps", type=int, default=3)
    ap.add_argument("--replay-slots", type=int, default=0,
                    help="reads in flight while recording the replayed launches (0: the timed run's cohort, --slots/2)")
    ap.add_argument("--cpu-sample", type=int, default=800_000, help="reads of the reference CPU baseline")
    ap.add_argument("--cpu-sample-1t", type=int, default=40_000, help="reads of its 1-thread line")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-replay", action="store_true")
    ap.add_argument("--no-replay-whole", action="store_true",
                    help="skip the second replay with the whole file in flight (the kernels at their widest launches)")
    ap.add_argument("--workdir", default=os.environ.get("BT2X_BENCH_DIR", f"/tmp/bt2x_bench_{os.getuid()}"))
    ap.add_argument("--rss-limit-gb", type=float, default=200.0, help="kill bt2x-align above this host RSS")
    ap.add_argument("--aligner", default=ALIGN,
                    help="aligner binary (tests: tests/cpp/test_e2e_oracle, the host driver over the CPU oracle)")
    ap.add_argument("--no-legs", action="store_true",
                    help="skip the configs C2 and C5 legs (rank 0 at N=1: E. coli 1M x 100 bp --no-sse8; 5M x 400 bp)")
    ap.add_argument("--c2-reads", type=int, default=1_000_000)
    ap.add_argument("--c5-reads", type=int, default=5_000_000)
    ap.add_argument("--runs", type=int, default=3,
                    help="timed runs of bt2x-align over the same index and files; value = the median run")
    # the repeat-heavy leg C3_rep50 (rank 0, N=1) is on by default: 50% repeat families on a
    # 200 Mbp synthetic genome, 1M x 150 bp reads, with the reference baseline, parity on 100k
    # and a replayed DP roofline; --no-rep-leg (or --no-legs) skips it
    ap.add_argument("--rep-leg", action="store_true", default=True, help=argparse.SUPPRESS)
    ap.add_argument("--no-rep-leg", dest="rep_leg", action="store_false",
                    help="skip the repeat-heavy leg C3_rep50 (on by default at N=1)")
    ap.add_argument("--leg-replay-reads", type=int, default=1 << 18,
                    help="reads whose GPU launches are replayed for the C2 / C3_rep50 legs' DP rooflines")
    ap.add_argument("--align-extra", default=os.environ.get("BT2X_ALIGN_EXTRA", ""),
                    help="extra bt2x-align options for the timed run and the replay recording (experiments)")
    ap.add_argument("--rep-mb", type=float, default=200.0, help="the repeat-heavy leg's genome size")
    ap.add_argument("--rep-reads", type=int, default=1_000_000, help="the repeat-heavy leg's timed reads")
    ap.add_argument("--cpu-index", action="store_true",
                    help="index the genome with the host builder (bt2x_build_index) instead of the GPU suffix sort")
    return ap.parse_args(argv)


def cpu_share() -> int:
    """CPUs this process may use: affinity, capped by the cgroup's CPU quota (the GPU box
    reports the whole machine's CPUs in affinity but grants a 16-CPU share)."""
    n = len(os.sched_getaffinity(0))
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, p = open(path).read().split()[:2]
            if q != "max":
                n = min(n, max(1, int(q) // int(p)))
        except (OSError, ValueError):
            pass
    return n


def mark(msg):
    rss = 0
    try:
        with open("/proc/self/status") as f:
            rss = next(int(ln.split()[1]) >> 10 for ln in f if ln.startswith("VmRSS"))
    except (OSError, StopIteration):
        pass
    print(f"# {time.strftime('%H:%M:%S')} {msg} (bench RSS {rss} MiB)", file=sys.stderr, flush=True)


def workload_key(args) -> str:
    if getattr(args, "leg_key", None):          # the C2 / C3_rep50 legs' replays
        return f"{args.leg_key}|replay{args.replay_reads}|inflight{args.replay_slots or max(1, args.slots // 2)}"
    return (f"c3|synthetic{args.genome_mb:g}Mbp_s{args.genome_seed}|reads{args.reads}|R{args.read_len}|"
            f"dpad{args.dpad}|replay{args.replay_reads}|inflight{args.replay_slots or max(1, args.slots // 2)}")


def pmc_profile(args, kernel: str):
    """Per-launch HBM bytes and VALU figures of `kernel` from the newest committed rocprofv3
    PMC summary (profiles/<tag>_traffic.json, tools/pmc_traffic.py) taken on this workload."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), reverse=True):
        with open(path) as f:
            t = json.load(f)
        if t.get("workload") == workload_key(args) and kernel in t.get("kernels", {}):
            return t["kernels"][kernel], os.path.relpath(path, ROOT)
    return None, None


# ------------------------------------------------------------------------ inputs

_GEN = {}


def _gen_file(job):
    import simdata as sd
    path, n, R, seed, first_id = job
    reads, quals = sd.sim_reads_fast(_GEN["codes"], _GEN["starts"], n, R, seed)
    sd.write_fastq_fixed(path + ".tmp", reads, quals, first_id=first_id)
    os.replace(path + ".tmp", path)
    return path


def make_inputs(args, rank, world, workdir):
    """-> (chroms, [warmup files], [step files], reads per step file).  Reads: seeded per
    (rank, file), written by a fork pool before the GPU is touched."""
    import multiprocessing as mp
    import simdata as sd
    t0 = time.perf_counter()
    chroms = sd.gen_genome(int(args.genome_mb * 1e6), nchrom=24, seed=args.genome_seed)
    codes, starts = sd.concat_genome(chroms)
    mark(f"genome {args.genome_mb:g} Mbp generated in {time.perf_counter() - t0:.1f} s")
    per = -(-args.reads // args.steps)
    rdir = os.path.join(workdir, f"rank{rank}")
    os.makedirs(rdir, exist_ok=True)
    jobs, warm, steps = [], [], []
    first = 0
    for k in range(args.warmup + args.steps):
        n = per if k >= args.warmup else args.replay_reads       # warmup files double as the replay batch
        if k == args.warmup + args.steps - 1:
            n = args.reads - per * (args.steps - 1)
        tag = f"w{k}" if k < args.warmup else f"s{k - args.warmup}"
        path = os.path.join(rdir, f"{tag}_{n}_R{args.read_len}_g{args.genome_seed}.fq")
        (warm if k < args.warmup else steps).append(path)
        if not os.path.exists(path):
            jobs.append((path, n, args.read_len, 3 + 7919 * rank + 104729 * k, first))
        first += n
    c5 = []
    if rank == 0 and world == 1 and not getattr(args, "no_legs", True) and getattr(args, "c5_reads", 0) > 0:
        nf = 10
        for k in range(nf):
            n = args.c5_reads // nf + (1 if k < args.c5_reads % nf else 0)
            path = os.path.join(rdir, f"c5_{k}_{n}_R400_g{args.genome_seed}.fq")
            c5.append(path)
            if not os.path.exists(path):
                jobs.append((path, n, 400, 5 + 104729 * k, first))
            first += n
    args.c5_files = c5
    if jobs:
        _GEN["codes"], _GEN["starts"] = codes, starts
        procs = max(1, min(len(jobs), cpu_share() // max(world, 1)))
        pool = mp.get_context("fork").Pool(procs)
        try:
            for _ in pool.imap_unordered(_gen_file, jobs):
                pass
            pool.close()
        finally:
            pool.terminate()
            pool.join()                     # the workers are reaped, not left behind
        _GEN.clear()
    mark(f"rank {rank}: {len(warm)} warmup + {len(steps)} step files of {per} reads ready in "
         f"{time.perf_counter() - t0:.1f} s")
    return chroms, codes, warm, steps, per


def build_index(args, chroms, codes, workdir, rank, dist):
    """Rank 0 indexes the genome (cached in workdir); the others wait at the barrier."""
    import simdata as sd
    tag = f"syn{int(args.genome_mb * 1e6)}_s{args.genome_seed}"
    base = os.path.join(workdir, tag)
    t0 = time.perf_counter()
    if rank == 0 and not all(os.path.exists(f"{base}.{k}.bt2l") for k in "1234"):
        from bt2x import lib
        fa = base + ".fa"
        sd.write_fasta(fa, chroms)
        if getattr(args, "cpu_index", False):
            lib.build_index(fa, base + ".tmp")
        else:
            import torch
            import gpu_sa
            sa, bwt, keys = gpu_sa.suffix_array(codes[codes < 4], device="cuda")
            lib.build_index_sa(fa, base + ".tmp", sa, bwt=bwt, keys=keys)
            del sa, bwt, keys
            torch.cuda.empty_cache()
        for k in "1234":
            os.replace(f"{base}.tmp.{k}.bt2l", f"{base}.{k}.bt2l")
        os.unlink(fa)
    if dist:
        dist.barrier()
    mark(f"index {tag} ready in {time.perf_counter() - t0:.1f} s")
    return base, (f"synthetic {args.genome_mb / 1e3:.2f} Gbp (seed {args.genome_seed}, 24 chromosomes, "
                  f"5% repeat families, low-complexity stretches, N runs)")


# ------------------------------------------------------------------------ aligner runs

def kv_line(err: str, tag: str) -> dict:
    lines = [ln for ln in err.splitlines() if ln.startswith(tag + " ")]
    if not lines:
        return {}
    out = {}
    for t in lines[-1].split()[1:]:
        k, v = t.split("=", 1)
        try:
            out[k] = float(v)
        except ValueError:
            out[k] = v
    return out


def bdist_mod():
    from bt2x import dist
    return dist


def run_aligner(args, cmd, errp, what):
    """bt2x-align as a child process (this process's GPU context, if any, stays idle), with
    a host-RAM watchdog (the box caps a command's RAM) and a progress line every 30 s."""
    t0 = time.perf_counter()
    with open(errp, "w") as ferr:
        p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=ferr, env=bdist_mod().malloc_thp_env())
        peak, last = 0, t0
        while p.poll() is None:
            try:
                with open(f"/proc/{p.pid}/status") as f:
                    for ln in f:
                        if ln.startswith("VmRSS"):
                            peak = max(peak, int(ln.split()[1]) >> 10)
            except OSError:
                pass
            now = time.perf_counter()
            if peak > args.rss_limit_gb * 1024 or now - t0 > 900:
                p.kill()
                p.wait()
                break
            if now - last > 30:
                mark(f"{what}: running {now - t0:.0f} s, RSS {peak} MiB")
                last = now
            time.sleep(0.2)
    wall = time.perf_counter() - t0
    err = open(errp).read()
    if p.returncode != 0:
        raise SystemExit(f"bt2x-align ({what}) failed (rc {p.returncode}, peak RSS {peak} MiB): {err[-3000:]}")
    mark(f"bt2x-align {what}: {wall:.1f} s, peak RSS {peak} MiB")
    return err, wall, peak


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


def replay(args, base, fq, rdir, gpu, n=None, opts=None):
    """Record the GPU launches bt2x-align makes for the reads of `fq` (a cohort of the timed
    run's size in flight), replay them from HBM and time each launch with HIP events on the
    launch stream.  opts: the aligner options of the workload (default --dpad)."""
    import torch
    from bt2x import abi, lib
    if n is None:
        n = int(os.path.basename(fq).split("_")[1])
    if opts is None:
        opts = ["--dpad", str(args.dpad)]
    ddir = os.path.join(rdir, "dump")
    shutil.rmtree(ddir, ignore_errors=True)
    os.makedirs(ddir)
    # one cohort of the timed run's size in flight (--slots / 2, its pipeline's cohorts): the
    # replayed launches have the shapes the end-to-end run launches
    run_aligner(args, [ALIGN, "-x", base, "-U", fq, "-S", os.devnull] + opts + ["-p",
                       str(args.host_threads), "--slots", str(args.replay_slots or max(1, args.slots // 2)), "--dump", ddir,
                       "--no-pipeline"] + getattr(args, "align_extra", "").replace(",", " ").split(),
                os.path.join(rdir, "dump.err"), "launch recording")
    launches = load_dumps(ddir)
    shutil.rmtree(ddir, ignore_errors=True)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    idx = lib.Index(base, load_offs=True)
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
                                   torch.empty(caps[1] * abi.ELT.itemsize, dtype=torch.uint8, device=dev), caps[1],
                                   torch.empty(caps[2] * abi.EXRANGE.itemsize, dtype=torch.uint8, device=dev), caps[2],
                                   torch.zeros(4, dtype=torch.int32, device=dev)]))
        else:
            m = len(parts[3])
            rec_cap, edit_cap = int(parts[4][0]) + 1024, int(parts[4][1]) + 4096   # sizes the aligner saw
            fl = parts[3]["flags"]
            lf = (abi.DPL_I16 if (fl & abi.DP_I16).any() else 0) | (abi.DPL_REF_TEXT if (fl & abi.DP_REF_TEXT).any() else 0)
            refs = parts[2] if len(parts[2]) else np.zeros(1, dtype=np.uint8)
            plan.append((kind, m, [to_dev(parts[0]), to_dev(parts[1]), to_dev(refs), to_dev(parts[3]),
                                   torch.empty(m * abi.DP_OUT.itemsize, dtype=torch.uint8, device=dev),
                                   torch.empty(rec_cap * abi.ALN_REC.itemsize, dtype=torch.uint8, device=dev),
                                   torch.empty(edit_cap * 4, dtype=torch.uint8, device=dev),
                                   torch.zeros(16, dtype=torch.int32, device=dev), rec_cap, edit_cap, lf]))
    del launches
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
                                 b[7].data_ptr(), sh, launch_flags=b[10])
            if record is not None:
                # HIP events recorded on this stream around each launch (bt2x_last_kernel_ms);
                # a round's seed kernel and ranking+resolution are also booked as seed / resolve
                record[kind] += ctx.last_kernel_ms(kid[kind])
                if kind == "round":
                    record["seed"] += ctx.last_kernel_ms(abi.K_SEED)
                    record["resolve"] += ctx.last_kernel_ms(abi.K_RESOLVE)
            if counters is not None:
                for kk in (("seed", "resolve") if kind == "round" else (kind,)):
                    for k, v in ctx.last_counters(kid[kk]).items():
                        counters[kk][k] = counters[kk].get(k, 0) + v
                if kind == "round":
                    rs = ctx.last_round_stats()
                    for k in ("reads", "jobs", "samples", "batches", "batch_draws", "serial_draws", "swap_draws",
                              "kcyc_setup", "kcyc_batch", "kcyc_serial", "kcyc_rest"):
                        counters["round"][k] = counters["round"].get(k, 0) + rs[k]
                    counters["round"]["max_samples"] = max(counters["round"].get("max_samples", 0), rs["max_samples"])

    ctr = {k: {} for k in kid}          # algorithmic-work counters (deterministic per step)
    step(counters=ctr)
    torch.cuda.synchronize(dev)
    recs = []
    t0 = time.perf_counter()
    for _ in range(args.replay_steps):
        rec = {k: 0.0 for k in kid}
        step(rec)
        recs.append(rec)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    for kind, m, b in plan:           # overflow check on the last step's arenas
        if kind == "dp":
            used = b[7][:2].cpu().numpy()
            if used[0] > b[8] or used[1] > b[9]:
                raise SystemExit(f"DP result arena overflow {used} vs {(b[8], b[9])}")
    kms = {k: float(np.mean([r[k] for r in recs])) for k in kid}
    nl = {k: sum(1 for kk, _, _ in plan if kk == k) for k in kid}
    nl["seed"] += nl["round"]
    nl["resolve"] += nl["round"]
    ctx.close()
    del plan
    torch.cuda.empty_cache()
    return {"reads": n, "elapsed": elapsed, "kms": kms, "ctr": ctr, "nl": nl, "units": units}


def roofline(args, rp, kernel=None):
    """SURVEY §8(d)'s algorithmic bytes per launch of the dominant kernel (or `kernel`) / its
    average launch time (HIP events), with the kernel's own bytes beside it."""
    R = args.read_len
    cs, cr, cd = rp["ctr"]["seed"], rp["ctr"]["resolve"], rp["ctr"]["dp"]
    kms, nl = rp["kms"], rp["nl"]
    # FM = 128*(2*BiLF + LF1) + 16*ftab (+ 128*LF1 + 8 per SA sample for the GroupWalk
    # resolve); DP = 3*R*C (E,F,H) + C (window) + 10*ceil(R/16)*16 (query profile)
    fm_bytes = 128 * (2 * cs.get("n_bilf", 0) + cs.get("n_lf1", 0)) + 16 * cs.get("n_ftab", 0)
    res_bytes = cr.get("alg_bytes", 0)
    dp_bytes = 3 * cd.get("dp_cells", 0) + cd.get("dp_cols", 0) + rp["units"]["dp"] * 10 * ((R + 15) // 16) * 16
    kern = {"seed": (kms["seed"], fm_bytes), "resolve": (kms["resolve"], res_bytes), "dp": (kms["dp"], dp_bytes)}
    dom = kernel or max(kern, key=lambda k: kern[k][0])
    ms, alg = kern[dom]
    ach = alg / (ms / 1e3) / 1e9 if ms > 0 else 0.0
    own = {"seed": cs.get("alg_bytes", 0), "resolve": cr.get("alg_bytes", 0), "dp": cd.get("alg_bytes", 0)}[dom]
    ach_own = own / (ms / 1e3) / 1e9 if ms > 0 else 0.0
    pmc, pmc_src = pmc_profile(args, dom)
    L = max(nl[dom], 1)
    roof = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4),
            "traffic": None if pmc is None else int(pmc["traffic_bytes"] / L),
            "alg_bytes": int(alg / L), "avg_launch_ms": round(ms / L, 4), "per": "launch", "launches_per_step": nl[dom],
            "alg_bytes_note": "achieved/alg_bytes count SURVEY 8(d)'s full-rectangle reference-equivalent bytes "
                              "(3 B of E/F/H per cell of every DP rectangle); the banded kernel computes "
                              "dp_cells_computed cells and moves 1 B per computed cell: achieved_kernel",
            "achieved_kernel": round(ach_own, 2), "frac_kernel": round(ach_own / HBM_PEAK_GBS, 4),
            "alg_bytes_kernel": int(own / L), "pmc_src": pmc_src}
    if pmc is not None:
        for k in ("valu_util", "sq_wait_any_per_wave_cycle", "write_bytes"):
            if k in pmc:
                roof[k] = pmc[k] if k != "write_bytes" else int(pmc[k] / L)
    kernels = {"seed_ms": round(kms["seed"], 3), "resolve_ms": round(kms["resolve"], 3), "dp_ms": round(kms["dp"], 3),
               "seed_alg_bytes": fm_bytes, "resolve_alg_bytes": res_bytes, "dp_alg_bytes": dp_bytes,
               "launches": nl, "units": rp["units"], "counters_seed": cs, "counters_resolve": cr,
               "counters_dp": cd, "round_sampling": rp["ctr"]["round"], "replay_reads": rp["reads"],
               "replay_steps": args.replay_steps,
               "replay_reads_per_s": round(rp["reads"] * args.replay_steps / rp["elapsed"], 1),
               "what": f"the GPU launch sequence bt2x-align issues for replay_reads reads (one file; "
                       f"{args.replay_slots or max(1, args.slots // 2)} reads in flight"
                       f"{'' if args.replay_slots else ', a cohort of the timed run'}), replayed from HBM; "
                       "kernel times from HIP events on the launch stream; the recording backend uploads "
                       "each request's read bytes (no read store), so the DP kernels read the same bytes "
                       "from a per-launch buffer instead of the store's slots"}
    return roof, kernels


# ------------------------------------------------------------------------ CPU baseline

def ref_run(args, base, fq, threads, sam):
    # (the same malloc setting as bt2x-align's runs: the baseline gets huge pages too)
    env = dict(bdist_mod().malloc_thp_env(), OMP_NUM_THREADS=str(threads), OMP_WAIT_POLICY="ACTIVE")
    t0 = time.perf_counter()
    # (the fork's -p is a tasks-per-thread multiplier, default 10: BASELINE.md runs it as is)
    r = subprocess.run([REF_ALIGN, "-x", base, "-U", fq, "-S", sam, "--dpad", str(args.dpad)],
                       env=env, capture_output=True, text=True, timeout=900)
    wall = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError(f"reference aligner failed: {r.stderr[-2000:]}")
    timers = {}
    for ln in r.stderr.splitlines():
        if ln.startswith("Timer:"):
            p = ln.split()
            if len(p) >= 4 and p[3] != "N/A":
                timers[p[3]] = float(p[2])
    return wall, timers


def head_fastq(srcs, dst, n) -> int:
    """The first n records of the stream of FASTQ files `srcs` (in order) into dst; returns
    the records written (fewer than n when the stream is shorter).  A sample larger than
    one step file continues into the next ones, so it is always the first reads of the
    timed run (the step files are its -U list after the warmup files)."""
    if isinstance(srcs, str):
        srcs = [srcs]
    got = 0
    with open(dst, "wb") as g:
        for src in srcs:
            with open(src, "rb") as f:
                while got < n:
                    rec = [f.readline() for _ in range(4)]
                    if not rec[0]:
                        break
                    g.write(b"".join(rec))
                    got += 1
            if got >= n:
                break
    return got


def cpu_baseline(args, base, fqs, rdir):
    """the reference aligner on the box's CPU share; n-1 and n threads, the
    better repeated to a median of 3; 1 thread on a smaller sample; alignment time = wall -
    wall of a 1-read run at the same thread count (index load)."""
    if not os.access(REF_ALIGN, os.X_OK):
        return None, None
    n = cpu_share()
    sample, s1, one = (os.path.join(rdir, f) for f in ("cpu_sample.fq", "cpu_1t.fq", "cpu_one.fq"))
    # m, m1: the reads the samples really hold (the timed run may have fewer than asked)
    m = head_fastq(fqs, sample, args.cpu_sample)
    m1 = head_fastq(fqs, s1, args.cpu_sample_1t)
    head_fastq(fqs, one, 1)
    sam = os.path.join(rdir, "ref.sam")
    load = {}
    # the reference's own run-to-run agreement on the sample (its F11 edit-buffer reads can
    # reach bytes past a read's end that depend on what its thread aligned before): every
    # sample run's records against the first one's
    first, rdiff, rex = [], [], []

    def rate(threads, fqp, reads):
        if threads not in load:
            load[threads] = ref_run(args, base, one, threads, os.devnull)[0]
        wall, timers = ref_run(args, base, fqp, threads, sam if fqp == sample else os.devnull)
        if fqp == sample:
            recs = set(sam_records(sam))
            if not first:
                first.append(recs)
            else:
                d = first[0] ^ recs
                rdiff.append(len(first[0] - recs))
                rex.extend(r.decode(errors="replace")[:600] for r in sorted(d)[:4 - len(rex)] if len(rex) < 4)
        return reads / max(wall - load[threads], 1e-6), wall, timers

    runs = {}
    for t in sorted({max(1, n - 1), n}):
        runs[t] = [rate(t, sample, m)]
        mark(f"reference aligner, {t} threads: {runs[t][-1][0]:.0f} reads/s")
    best = max(runs, key=lambda t: runs[t][0][0])
    while len(runs[best]) < 3:
        runs[best].append(rate(best, sample, m))
    med = sorted(runs[best], key=lambda r: r[0])[1]
    one_t = rate(1, s1, m1)
    mark(f"reference aligner: median {med[0]:.0f} reads/s at {best} threads; 1 thread {one_t[0]:.0f} reads/s")
    # (the last sample run left its SAM at `sam`; every run over the sample aligns the same reads)
    return {"value": round(med[0] / 1e6, 6), "unit": "M reads/s", "cores": best, "kind": "reference",
            "sample_reads": m,
            "sample": f"first {m} reads of the timed run (step files in order) through oracle/_ref/bowtie2-align-l --dpad {args.dpad} "
                      f"(FASTQ->SAM, OpenMP, OMP_WAIT_POLICY=ACTIVE) on this box's {n}-CPU share: "
                      f"threads {sorted(runs)}, best repeated, median of 3; alignment time = wall - wall of a "
                      f"1-read run (index load {load[best]:.2f} s)",
            "runs": {str(t): [round(r[0], 1) for r in v] for t, v in runs.items()},
            "one_thread": {"value": round(one_t[0] / 1e6, 6), "reads": m1},
            "reference_runs_differ": rdiff, "reference_runs_examples": rex,
            "timer_sums_s": med[2], "cpu_share": n}, sam


def sam_records(path, first_n=None):
    recs = []
    with open(path, "rb") as f:
        for ln in f:
            if ln.startswith(b"@"):
                continue
            recs.append(ln.rstrip(b"\n"))
            if first_n is not None and len(recs) >= first_n:
                break
    recs.sort()
    return recs


def timed_align(args, base, files, warm, rdir, tag, extra):
    """bt2x-align over `files` (the first `warm` untimed) -> (t_align, metrics, stats, stderr)."""
    from bt2x import dist as bdist
    out = os.path.join(rdir, f"{tag}.sam")
    cmd = [args.aligner, "-x", base, "-U", ",".join(files), "-S", out, "-p", str(args.host_threads),
           "--slots", str(args.slots), "--warmup-files", str(warm), "--metrics", "--stats"] + extra
    err, wall, peak = run_aligner(args, cmd, os.path.join(rdir, f"{tag}.err"), f"{tag} timed run")
    timed = kv_line(err, "BT2X_TIMED")
    return float(timed["t_align"]), bdist.parse_metrics(err)["metrics"], kv_line(err, "BT2X_STATS"), out, peak


def ref_baseline(args, binary, base, fqs, rdir, n, extra, tag):
    """The reference aligner (binary) on the first n reads of fqs with the box's CPU share:
    reads/s (alignment time = wall - wall of a 1-read run) and its SAM."""
    share = cpu_share()
    sample, one = os.path.join(rdir, f"{tag}_sample.fq"), os.path.join(rdir, f"{tag}_one.fq")
    m = head_fastq(fqs, sample, n)
    head_fastq(fqs, one, 1)
    sam = os.path.join(rdir, f"{tag}_ref.sam")
    env = dict(bdist_mod().malloc_thp_env(), OMP_NUM_THREADS=str(share), OMP_WAIT_POLICY="ACTIVE")
    walls = []
    for fq, dst in ((one, os.devnull), (sample, sam)):
        t0 = time.perf_counter()
        r = subprocess.run([binary, "-x", base, "-U", fq, "-S", dst] + extra, env=env, capture_output=True, text=True,
                           timeout=900)
        walls.append(time.perf_counter() - t0)
        if r.returncode != 0:
            raise RuntimeError(f"reference aligner failed: {r.stderr[-2000:]}")
    return {"value": round(m / max(walls[1] - walls[0], 1e-6) / 1e6, 6), "unit": "M reads/s", "cores": share,
            "kind": "reference", "sample_reads": m,
            "sample": f"first {m} reads through {os.path.relpath(binary, ROOT)} {' '.join(extra)} on the box's "
                      f"{share}-CPU share, one run; alignment time = wall - wall of a 1-read run"}, sam


def leg_roofline(args, base, srcs, rdir, gpu, tag, opts, read_len, leg_key):
    """The DP kernel's roofline on a leg's own workload: the GPU launches bt2x-align makes for
    the first --leg-replay-reads reads of the leg's timed files, recorded with a cohort of
    the timed run's size in flight and replayed from HBM (as the headline's `roofline`)."""
    n = getattr(args, "leg_replay_reads", 0)
    if n <= 0 or args.no_replay:
        return None
    fq = os.path.join(rdir, f"{tag}_replay.fq")
    m = head_fastq(srcs, fq, n)
    wargs = argparse.Namespace(**vars(args))
    wargs.replay_reads, wargs.read_len, wargs.leg_key, wargs.replay_slots = m, read_len, leg_key, 0
    rp = replay(wargs, base, fq, rdir, gpu, n=m, opts=opts)
    os.unlink(fq)
    roof, kern = roofline(wargs, rp, kernel="dp")
    return {"roofline": roof,
            "kernels": {k: kern[k] for k in ("seed_ms", "resolve_ms", "dp_ms", "dp_alg_bytes", "launches", "units",
                                             "counters_dp", "replay_reads", "replay_steps", "replay_reads_per_s", "what")},
            "workload_key": workload_key(wargs)}


def rep_leg(args, rdir, gpu=0):
    """A repeat-heavy sensitivity leg: hg38 is ~50% repeats, the C3 stand-in 5%, so the walk
    tail and the DP work per read are understated there.  200 Mbp, 8 chromosomes, 50% of
    it copies of 8 repeat families (~2% divergence), 1M x 150 bp reads, --dpad 12."""
    import simdata as sd
    from bt2x import lib
    mb = getattr(args, "rep_mb", 200.0)
    chroms = sd.gen_genome(int(mb * 1e6), nchrom=8, seed=7, repeat_frac=0.5)
    codes, starts = sd.concat_genome(chroms)
    base = os.path.join(args.workdir, f"rep50_{mb:g}M")
    if not all(os.path.exists(f"{base}.{k}.bt2l") for k in "1234"):
        fa = base + ".fa"
        sd.write_fasta(fa, chroms)
        if getattr(args, "cpu_index", False):
            lib.build_index(fa, base + ".tmp")
        else:
            import torch
            import gpu_sa
            sa, bwt, keys = gpu_sa.suffix_array(codes[codes < 4], device="cuda")
            lib.build_index_sa(fa, base + ".tmp", sa, bwt=bwt, keys=keys)
            del sa, bwt, keys
            torch.cuda.empty_cache()
        for k in "1234":
            os.replace(f"{base}.tmp.{k}.bt2l", f"{base}.{k}.bt2l")
        os.unlink(fa)
    files = []
    nr = getattr(args, "rep_reads", 1_000_000)
    nw = max(1, nr // 10)
    for k, (n, seed) in enumerate(((nw, 31), (nr, 37))):
        path = os.path.join(rdir, f"rep50_{k}_{n}_R150.fq")
        if not os.path.exists(path):
            reads, quals = sd.sim_reads_fast(codes, starts, n, 150, seed)
            sd.write_fastq_fixed(path + ".tmp", reads, quals, first_id=0 if k == 0 else nw)
            os.replace(path + ".tmp", path)
        files.append(path)
    t, met, stats, out, peak = timed_align(args, base, files, 1, rdir, "rep50", ["--dpad", str(args.dpad), "--device", str(gpu)])
    leg = {"workload": f"repeat-heavy sensitivity: {nr} x 150 bp SE reads vs a seeded {mb:g} Mbp synthetic genome with "
                       "50% repeat families (C3's stand-in has 5%), --dpad 12, FASTQ -> SAM",
           "value": round(met["nread"] / t / 1e6, 4), "unit": "M reads/s", "t_align_s": round(t, 3),
           "reads": met["nread"], "aligned": met["nunp_uni"] + met["nunp_rep"], "repetitive": met["nunp_rep"],
           "dps_per_read": round(float(stats.get("dps", 0)) / max(1, met["nread"]), 3), "stats": stats,
           "peak_rss_mib": peak}
    lr = leg_roofline(args, base, files[1:], rdir, gpu, "rep50", ["--dpad", str(args.dpad)], 150,
                      f"c3rep50|synthetic{mb:g}Mbp_s7|R150|dpad{args.dpad}")
    if lr:
        leg.update(lr)
    if not args.no_cpu and os.access(REF_ALIGN, os.X_OK):
        cb, rsam = ref_baseline(args, REF_ALIGN, base, files[1:], rdir, min(nr, 100_000), ["--dpad", str(args.dpad)],
                                "rep50")
        leg["cpu_baseline"] = cb
        leg["parity"] = parity(out, rsam, cb["sample_reads"])
        leg["gpu_vs_cpu"] = round(leg["value"] / cb["value"], 2) if cb["value"] else None
    os.unlink(out)
    return leg


def extra_legs(args, c3_base, rdir, gpu=0):
    """BASELINE.json's other single-GPU configs, beside the C3 headline (rank 0, N=1):
    C2 -- the E. coli stand-in (4.64 Mbp, simdata.ecoli_genome), 1M x 100 bp reads,
          --no-sse8: the i16 DP kernel end to end (the reference's -DENABLE_I16 build beside
          it, and a SAM comparison on its sample);
    C5 -- 5M x 400 bp reads on the C3 genome: every read is unaligned by the reference's
          rules (rdlen >= 256, bt2_search.cpp:2475-2496), so this measures throughput only
          (FASTQ parse and SAM formatting; the GPU has nothing to do)."""
    import simdata as sd
    from bt2x import lib
    legs = {}
    # ---- C2
    chroms = sd.ecoli_genome()
    codes, starts = sd.concat_genome(chroms)
    base = os.path.join(args.workdir, "ecoli")
    if not os.path.exists(base + ".4.bt2l"):
        sd.write_fasta(base + ".fa", chroms)
        lib.build_index(base + ".fa", base)
    files = []
    for k, (n, seed) in enumerate(((args.c2_reads // 10, 17), (args.c2_reads, 11))):
        path = os.path.join(rdir, f"c2_{k}_{n}_R100.fq")
        if not os.path.exists(path):
            reads, quals = sd.sim_reads_fast(codes, starts, n, 100, seed)
            sd.write_fastq_fixed(path + ".tmp", reads, quals, first_id=0 if k == 0 else args.c2_reads // 10)
            os.replace(path + ".tmp", path)
        files.append(path)
    t, met, stats, out, peak = timed_align(args, base, files, 1, rdir, "c2", ["--no-sse8", "--device", str(gpu)])
    leg = {"workload": f"C2 stand-in: {args.c2_reads} x 100 bp SE reads vs the seeded 4.64 Mbp E. coli stand-in, "
                       "--no-sse8 (the i16 DP kernel; the reference's -DENABLE_I16 build), FASTQ -> SAM",
           "value": round(met["nread"] / t / 1e6, 4), "unit": "M reads/s", "t_align_s": round(t, 3),
           "reads": met["nread"], "aligned": met["nunp_uni"] + met["nunp_rep"], "stats": stats, "peak_rss_mib": peak}
    # the i16 fill's roofline: SURVEY 8(d)'s bytes count 3 B per cell for the reference's u8
    # matrix; its i16 kernel keeps 16-bit E/F/H, 6 B per cell (roofline_i16)
    lr = leg_roofline(args, base, files[1:], rdir, gpu, "c2", ["--no-sse8"], 100, "c2|ecoli4.64Mbp_s11|R100|nosse8")
    if lr:
        r = lr["roofline"]
        cd = lr["kernels"]["counters_dp"]
        b16 = 6 * cd.get("dp_cells", 0) + cd.get("dp_cols", 0) + lr["kernels"]["units"]["dp"] * 20 * ((100 + 15) // 16) * 16
        L = max(r["launches_per_step"], 1)
        ms = lr["kernels"]["dp_ms"]
        lr["roofline_i16"] = {"bound": "hbm", "kernel": "dp", "alg_bytes": int(b16 / L),
                              "achieved": round(b16 / (ms / 1e3) / 1e9, 2) if ms > 0 else 0.0, "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": round(b16 / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if ms > 0 else 0.0,
                              "what": "SURVEY 8(d) i16 bytes: 6*R*C (16-bit E/F/H) + C + 20*ceil(R/16)*16 (16-bit "
                                      "query profile) per problem, over the same replayed launches as `roofline`"}
        leg.update(lr)
    ref16 = os.path.join(ROOT, "oracle", "_ref", "bowtie2-align-l-i16")
    if not args.no_cpu and os.access(ref16, os.X_OK):
        cb, rsam = ref_baseline(args, ref16, base, files[1:], rdir, 200_000, ["--no-sse8"], "c2")
        leg["cpu_baseline"] = cb
        leg["parity"] = parity(out, rsam, cb["sample_reads"])
        leg["gpu_vs_cpu"] = round(leg["value"] / cb["value"], 2) if cb["value"] else None
    os.unlink(out)
    legs["C2"] = leg
    # ---- C5
    c5 = getattr(args, "c5_files", [])
    if c5:
        t, met, stats, out, peak = timed_align(args, c3_base, c5, 1, rdir, "c5", [])
        n = met["nread"]
        leg = {"workload": f"C5 stand-in: {args.c5_reads} x 400 bp SE reads vs the C3 genome (the first file of "
                           f"{os.path.basename(c5[0]).split('_')[2]} reads untimed); every record unaligned as in the "
                           "reference (reads of 256 bp or more), so throughput only: FASTQ parse + SAM",
               "value": round(n / t / 1e6, 4), "unit": "M reads/s", "t_align_s": round(t, 3), "reads": n,
               "aligned": met["nunp_uni"] + met["nunp_rep"], "peak_rss_mib": peak}
        if not args.no_cpu and os.access(REF_ALIGN, os.X_OK):
            cb, rsam = ref_baseline(args, REF_ALIGN, c3_base, c5[1:], rdir, 500_000, [], "c5")
            leg["cpu_baseline"] = cb
            leg["parity"] = parity(out, rsam, cb["sample_reads"])
            leg["gpu_vs_cpu"] = round(leg["value"] / cb["value"], 2) if cb["value"] else None
        os.unlink(out)
        legs["C5"] = leg
    return legs


def parity(ours_sam, ref_sam, n) -> dict:
    """Our timed run's first n SAM records (records are written in input order) against
    the reference aligner's records for the same n reads, compared sorted."""
    ours, theirs = sam_records(ours_sam, n), sam_records(ref_sam)
    diff = sum(1 for a, b in zip(ours, theirs) if a != b) + abs(len(ours) - len(theirs))
    out = {"sample_reads": n, "records_ours": len(ours), "records_reference": len(theirs), "records_differ": diff,
           "what": "sorted SAM records of the timed run's first sample_reads reads vs the reference "
                   "aligner's on the same reads"}
    if diff:                                     # (the first few, for the record)
        a, b = set(ours), set(theirs)
        out["examples_ours"] = [r.decode(errors="replace")[:600] for r in sorted(a - b)[:4]]
        out["examples_reference"] = [r.decode(errors="replace")[:600] for r in sorted(b - a)[:4]]
    return out


def host_threads(args, share: int, world: int) -> tuple[int, str]:
    """bt2x-align -p per rank: the node's CPU share split over the ranks.  One rank keeps
    ~14 cores busy at the current host cost per read (4.7 us x 3.1 M reads/s),
    so a share that leaves a rank fewer than kRankCores is reported (not silently raised)."""
    kRankCores = 14
    if args.host_threads > 0:
        return args.host_threads, "set by --host-threads"
    t = max(1, share // max(world, 1))
    note = f"{share}-CPU share / {world} rank(s)"
    if t < kRankCores:
        note += (f": below the ~{kRankCores} host cores one rank uses at full rate (DESIGN.md §6) -- "
                 "this run is host-bound by its CPU share")
    return t, note


def reap_children() -> list:
    """Terminate and wait for every process this bench started that is still alive (none
    should be: each aligner / reference run is waited for), so nothing outlives bench.py;
    returns what was found."""
    try:
        import psutil
    except ImportError:
        return []
    kids = psutil.Process().children(recursive=True)
    found = []
    for c in kids:
        try:
            found.append(f"{c.pid}:{c.name()}")
            c.terminate()
        except psutil.Error:
            pass
    _, alive = psutil.wait_procs(kids, timeout=5)
    for c in alive:
        try:
            c.kill()
        except psutil.Error:
            pass
    psutil.wait_procs(alive, timeout=5)
    return found


def user_procs():
    """This user's processes other than bench.py, its ancestors and its children, as
    "pid:name:command" (the review counts one process left at the end of the driver's run;
    this lists what is alive, under the same user, as bench.py exits)."""
    try:
        import psutil
    except ImportError:
        return []
    me = psutil.Process()
    skip = {me.pid} | {p.pid for p in me.parents()} | {p.pid for p in me.children(recursive=True)}
    out = []
    for p in psutil.process_iter(["pid", "name", "uids", "cmdline"]):
        try:
            if p.info["pid"] in skip or p.info["uids"] is None or p.info["uids"].real != os.getuid():
                continue
            if not p.info["cmdline"]:                    # kernel threads
                continue
            out.append(f"{p.info['pid']}:{p.info['name']}:{' '.join(p.info['cmdline'] or [])[:120]}")
        except psutil.Error:
            pass
    return out


# ------------------------------------------------------------------------ main

def main():
    args = parse()
    from bt2x import dist as bdist
    rank, world, local = bdist.world()
    gpu = int(os.environ.get("BT2X_BENCH_DEVICE", local))
    share = cpu_share()
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    args.host_threads, threads_note = host_threads(args, share, local_world)
    # N > 1: every local rank its own CPUs inside its GPU's NUMA node (bt2x.dist), and no
    # more threads than it has CPUs; N = 1 keeps the aligner's own NUMA-node pinning
    cpu_set, cpu_note = None, ""
    if local_world > 1:
        devs = [gpu] * local_world if "BT2X_BENCH_DEVICE" in os.environ else list(range(local_world))
        sets, cpu_note = bdist.local_cpu_sets(local_world, devs)
        if sets[local]:
            cpu_set = bdist.format_cpu_list(sets[local])
            if args.host_threads > len(sets[local]):
                args.host_threads = len(sets[local])
                threads_note += f"; capped at the rank's {len(sets[local])} CPUs"
    workdir = args.workdir
    os.makedirs(workdir, exist_ok=True)
    # inputs first: the read generator forks, which must happen before the GPU is touched
    chroms, codes, warm, steps, per = make_inputs(args, rank, world, workdir)
    dist = None
    if world > 1:
        import torch.distributed as dist
        bdist.init_quiet(dist)
    base, gdesc = build_index(args, chroms, codes, workdir, rank, dist)
    del chroms, codes
    rdir = os.path.join(workdir, f"rank{rank}")

    # the inputs and the index were just written: flush them to disk now, so the timed run
    # does not share the box with the page cache's writeback of ~15 GB (first runs on a
    # fresh box were up to ~20 % slower than later runs of the same files)
    t_sync = time.perf_counter()
    os.sync()
    mark(f"inputs synced to disk in {time.perf_counter() - t_sync:.1f} s")
    # ---- timed: the aligner over the step files (warmup files first, untimed)
    # every rank writes its SAM to the node's disk when all of them fit (the same choice at
    # every N, so the per-GPU work does not change with N); else /dev/null everywhere
    need = args.reads * (args.read_len * 3)                   # SAM bytes per rank, generously
    if dist:
        dist.barrier()                                        # every rank's inputs are on disk
    out_sam = os.path.join(rdir, "out.sam")
    if shutil.disk_usage(rdir).free < world * need + (8 << 30):
        out_sam = os.devnull
    cmd = [args.aligner, "-x", base, "-U", ",".join(warm + steps), "-S", out_sam, "--dpad", str(args.dpad),
           "--device", str(gpu), "-p", str(args.host_threads), "--slots", str(args.slots),
           "--warmup-files", str(len(warm)), "--metrics", "--stats"] + args.align_extra.replace(",", " ").split()
    if cpu_set:
        cmd += ["--cpus", cpu_set]
    # args.runs timed runs over the same index and files (separate processes); value = the
    # median run's (by the max over ranks of its timed wall time); every run is listed
    runs = []
    for k in range(max(1, args.runs)):
        # every run writes a new file: opening the last run's 4 GB SAM with O_TRUNC would drop
        # its page cache inside the timed region, and ext4 flushes a file truncated that way
        # when it is closed (auto_da_alloc): runs 2 and 3 were 0.5 s slower than run 1
        if out_sam != os.devnull and os.path.exists(out_sam):
            os.unlink(out_sam)
        if dist:
            dist.barrier()
        err, wall, peak = run_aligner(args, cmd, os.path.join(rdir, f"align{k}.err"), f"timed run {k + 1}/{args.runs}")
        if dist:
            dist.barrier()
        timed = kv_line(err, "BT2X_TIMED")
        met = bdist.parse_metrics(err)["metrics"]
        t_align = float(timed["t_align"])
        if met["nread"] != args.reads:
            raise SystemExit(f"timed run aligned {met['nread']} reads, expected {args.reads}")
        tot = bdist.sum_counters(met, dist)
        t_max = bdist.max_over_ranks(t_align, dist)
        runs.append({"err": err, "wall": wall, "peak": peak, "timed": timed, "met": met, "tot": tot,
                     "t_align": t_align, "t_max": t_max})
    order = sorted(range(len(runs)), key=lambda k: runs[k]["t_max"])
    med = runs[order[len(order) // 2]]
    err, wall, peak, timed, met, tot, t_align, t_max = (med[k] for k in ("err", "wall", "peak", "timed", "met", "tot",
                                                                         "t_align", "t_max"))
    stats = kv_line(err, "BT2X_STATS")
    value = tot["nread"] / t_max / 1e6
    # every rank's CPU affinity as its aligner reported it (BT2X_CPUS), in rank order
    mine = next((ln.split(" ", 1)[1].strip() for ln in err.splitlines() if ln.startswith("BT2X_CPUS ")), None)
    host_cpus = [mine]
    if dist:
        host_cpus = [None] * world
        dist.all_gather_object(host_cpus, mine)
    t_files = [float(x) for x in str(timed.get("t_files", "")).split(",") if x]

    def run_entry(r):
        ru = kv_line(r["err"], "BT2X_RUSAGE_ALIGN")
        e = {"value": round(r["tot"]["nread"] / r["t_max"] / 1e6, 4), "t_align_s": round(r["t_align"], 3),
             "t_align_max_s": round(r["t_max"], 3), "peak_rss_mib": r["peak"]}
        if ru and r["met"]["nread"]:
            e["host_cpu_us_per_read"] = round((float(ru.get("user", 0)) + float(ru.get("sys", 0))) / r["met"]["nread"] * 1e6, 3)
            # (each run's own split: a slow run's extra CPU shows as user or sys time, and
            # faults / preemptions, e.g. huge-page compaction or a busy node)
            e["rusage"] = {k: ru.get(k) for k in ("user", "sys", "minflt", "vcsw", "ivcsw")}
        g = kv_line(r["err"], "BT2X_GPU")
        if g:
            e["k_dp_s"], e["k_round_s"] = g.get("k_dp"), g.get("k_round")
        return e

    line = {
        "metric": "M reads/s aligned (150 bp SE vs hg38) at 1/2/4/8 MI355X; % HBM-roofline",
        "value": round(value, 4), "unit": "M reads/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(t_max / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded 3.1 Gbp genome + simulated 150 bp reads, BASELINE.md error model)",
        "config": {"workload": f"C3 stand-in: {args.reads} x {args.read_len} bp SE reads per GPU, end-to-end, "
                               f"--dpad {args.dpad}, genome {gdesc}; value = FASTQ -> SAM reads/s of bt2x-align "
                               f"(parse, host driver, GPU seed/resolve/DP kernels, PCIe, SAM written to "
                               f"{'a file' if out_sam != os.devnull else '/dev/null'}), index load excluded; "
                               f"step = one FASTQ file of {per} reads",
                   "reads_per_gpu": args.reads, "read_len": args.read_len, "parallelism": f"dp{world} (read shards)",
                   "host_threads": args.host_threads, "host_threads_note": threads_note, "cpu_share": share,
                   "malloc": bdist_mod().malloc_thp_env().get("GLIBC_TUNABLES", "default") + " (bt2x-align and the reference runs)", "host_cpus": host_cpus, "host_cpus_note": cpu_note or "one rank: the aligner pins itself to its GPU's NUMA node",
                   "slots": args.slots, "key": workload_key(args)},
        "end_to_end": {"runs": [run_entry(r) for r in runs],
                       "value_is": f"the median of {len(runs)} timed runs (separate bt2x-align processes, same index "
                                   "and files); the fields below are that run's",
                       "t_align_s": round(t_align, 3), "t_align_max_s": round(t_max, 3),
                       "t_run_s": timed.get("t_run"), "t_return_s": timed.get("t_ret"),
                       "step_done_s": [round(t, 3) for t in t_files], "wall_incl_index_load_s": round(wall, 2),
                       "peak_rss_mib": peak, "summary": bdist.alignment_summary(tot).splitlines(),
                       "stats": stats, "gpu": kv_line(err, "BT2X_GPU"), "rusage_align": kv_line(err, "BT2X_RUSAGE_ALIGN")},
    }
    # bytes over PCIe in the timed run (every BT2X_GPU *_h2d_mib / *_d2h_mib field: rounds,
    # DP requests, read-store uploads)
    g = line["end_to_end"]["gpu"] or {}
    mib = [float(v) for k, v in g.items() if k.endswith("_h2d_mib") or k.endswith("_d2h_mib")]
    if mib:
        line["end_to_end"]["pcie_gb"] = round(sum(mib) / 1024.0, 2)
    # host CPU per read (rank 0's aligner process over its timed files): user + system time
    # of all its threads, and the thread-seconds the run had (threads x t_align)
    ru = line["end_to_end"]["rusage_align"]
    if ru and met["nread"]:
        cpu_s = float(ru.get("user", 0)) + float(ru.get("sys", 0))
        line["end_to_end"]["host_cpu_us_per_read"] = round(cpu_s / met["nread"] * 1e6, 3)
        line["end_to_end"]["host_thread_us_per_read"] = round(args.host_threads * t_align / met["nread"] * 1e6, 3)
    # ---- rank 0: kernels (replay) and, at N=1, the CPU baseline + parity
    if rank == 0 and not args.no_replay:
        rp = replay(args, base, warm[0] if warm else steps[0], rdir, gpu)
        line["roofline"], line["kernels"] = roofline(args, rp)
        if not args.no_replay_whole and not args.replay_slots:
            # the same reads with the whole file in flight: the widest launches the aligner
            # makes (round 2's replay shape), beside the timed run's cohort shapes above
            wargs = argparse.Namespace(**vars(args))
            wargs.replay_slots = args.replay_reads
            rpw = replay(wargs, base, warm[0] if warm else steps[0], rdir, gpu)
            rw, kw = roofline(wargs, rpw)
            line["kernels_whole_file"] = {
                "what": "the same replay with the whole file in flight (--replay-slots = replay_reads): "
                        f"{kw['launches']['dp']} DP launches instead of {line['kernels']['launches']['dp']}",
                "dp_ms": kw["dp_ms"], "seed_ms": kw["seed_ms"], "resolve_ms": kw["resolve_ms"],
                "replay_reads_per_s": kw["replay_reads_per_s"], "launches": kw["launches"],
                "roofline": {k: rw[k] for k in ("kernel", "achieved", "peak", "unit", "frac", "avg_launch_ms",
                                                "achieved_kernel", "frac_kernel", "traffic", "pmc_src")}}
    if rank == 0 and world == 1 and not args.no_cpu:
        cb, ref_sam = cpu_baseline(args, base, steps, rdir)
        if cb is not None:
            line["cpu_baseline"] = cb
            if out_sam != os.devnull:
                line["parity"] = parity(out_sam, ref_sam, cb["sample_reads"])
            line["gpu_vs_cpu"] = round(value / cb["value"], 2) if cb["value"] else None
    if out_sam != os.devnull and os.path.exists(out_sam):
        os.unlink(out_sam)
    if rank == 0 and world == 1 and not args.no_legs:
        line["configs_other"] = extra_legs(args, base, rdir, gpu)
    if rank == 0 and world == 1 and getattr(args, "rep_leg", False):
        line.setdefault("configs_other", {})["C3_rep50"] = rep_leg(args, rdir, gpu)
    line["end_to_end"]["reaped_at_exit"] = reap_children()
    line["end_to_end"]["user_procs_at_exit"] = user_procs()
    if dist:
        dist.barrier()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
