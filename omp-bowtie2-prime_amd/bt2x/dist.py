"""Read sharding across GPUs: one process per GPU, the index replicated
in every GPU's HBM, reads partitioned, no collective on the data path.

Every read is independent and its RNG stream is derived from its own content
(pat.cpp:45-88), so any read-to-rank assignment gives the same per-read results; the
only cross-rank step is the final sum of the additive counters (ReportingMetrics,
aln_sink.h:148) and, for the benchmark, the max of the ranks' wall times.
"""
from __future__ import annotations

import os


def init_quiet(dist, backend: str = "gloo") -> None:
    """dist.init_process_group(backend) with the backend's connection chatter ("[Gloo] Rank
    0 is connected to ...", written to fd 1 by the C++ side) kept off stdout, where the
    bench's one JSON line and SAM output go."""
    import sys
    sys.stdout.flush()
    saved = os.dup(1)
    null = os.open(os.devnull, os.O_WRONLY)
    try:
        os.dup2(null, 1)
        dist.init_process_group(backend)
        dist.barrier()
    finally:
        os.dup2(saved, 1)
        os.close(saved)
        os.close(null)


def world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_bounds(n: int, rank: int, world_size: int) -> tuple[int, int]:
    """Contiguous, balanced [lo, hi) slice of n reads for `rank` (sizes differ by <= 1)."""
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError(f"bad rank {rank} of {world_size}")
    q, r = divmod(n, world_size)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def rank_seed(base_seed: int, rank: int) -> int:
    """Per-rank seed of the synthetic read batch (weak scaling: every rank its own batch)."""
    return base_seed + 7919 * rank


def sum_counters(counters: dict, dist=None, device=None) -> dict:
    """Sum integer counters over ranks (the one reduction the path needs)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return dict(counters)
    import torch
    keys = sorted(counters)
    t = torch.tensor([int(counters[k]) for k in keys], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return {k: int(v) for k, v in zip(keys, t.tolist())}


def max_over_ranks(x: float, dist=None, device=None) -> float:
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(x)
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# ---------------------------------------------------------------- sharded aligner runs
#
# python -m torch.distributed.run --nproc-per-node N -m bt2x.dist [--aligner PATH] -- \
#     <bt2x-align arguments, including -S out.sam>
#
# Each rank runs the aligner as a child process on its own GPU (HIP_VISIBLE_DEVICES =
# LOCAL_RANK; this process never touches the GPU) over shard RANK/N of the read stream
# (bt2x-align --shard, FastqReader), writing out.sam.part<RANK>.  The ranks then sum the
# 27 ReportingMetrics counters (gloo all-reduce: the only collective; bt2_search.cpp:
# 2867-2869 is the reference's per-thread merge of the same counters), rank 0 appends
# the parts in rank order to out.sam -- the single run's SAM, as the shards are
# contiguous and in order -- and prints the reference's alignment summary of the sum.

METRIC_NAMES = (
    "nread", "npaired", "nunpaired", "nconcord_uni", "nconcord_uni1", "nconcord_uni2", "nconcord_rep",
    "nconcord_0", "ndiscord", "nunp_0_uni", "nunp_0_uni1", "nunp_0_uni2", "nunp_0_rep", "nunp_0_0",
    "nunp_rep_uni", "nunp_rep_uni1", "nunp_rep_uni2", "nunp_rep_rep", "nunp_rep_0", "nunp_uni", "nunp_uni1",
    "nunp_uni2", "nunp_rep", "nunp_0", "sum_best1", "sum_best2", "sum_best")   # aln_sink.h:44-170


def parse_metrics(text: str) -> dict:
    """The aligner's BT2X_METRICS (27 counters) and BT2X_TIMED lines from its stderr."""
    met, timed = None, {}
    for ln in text.splitlines():
        if ln.startswith("BT2X_METRICS "):
            vals = [int(v) for v in ln.split()[1:]]
            if len(vals) != len(METRIC_NAMES):
                raise ValueError(f"BT2X_METRICS has {len(vals)} fields, expected {len(METRIC_NAMES)}")
            met = dict(zip(METRIC_NAMES, vals))
        elif ln.startswith("BT2X_TIMED "):
            for kv in ln.split()[1:]:
                k, v = kv.split("=", 1)
                timed[k] = v
    if met is None:
        raise ValueError("aligner printed no BT2X_METRICS line")
    return {"metrics": met, "timed": timed}


def alignment_summary(m: dict) -> str:
    """AlnSink::printAlSumm for unpaired reads with -M's repetitive threshold (aln_sink.cpp:349-527)."""
    def pct(a, b):
        return f"{100.0 * a / b if b else 0.0:.2f}%"
    nread, nun = m["nread"], m["nunpaired"]
    out = [f"{nread} reads; of these:" if nread else f"{nread} reads"]
    if nun:
        more = m["nunp_uni2"] + m["nunp_rep"]
        out += [f"  {nun} ({pct(nun, nread)}) were unpaired; of these:",
                f"    {m['nunp_0']} ({pct(m['nunp_0'], nun)}) aligned 0 times",
                f"    {m['nunp_uni1']} ({pct(m['nunp_uni1'], nun)}) aligned exactly 1 time",
                f"    {more} ({pct(more, nun)}) aligned >1 times"]
    out.append(f"{pct(m['nunp_uni'] + m['nunp_rep'], nun)} overall alignment rate")
    return "\n".join(out) + "\n"


def rank_device(local_rank: int, env=None) -> str:
    """The GPU of local rank k: the k-th entry of an existing HIP_VISIBLE_DEVICES (or
    ROCR_VISIBLE_DEVICES) mask, so a job launched on a subset of a node's GPUs stays on
    it; the k-th GPU of the node when neither is set."""
    env = os.environ if env is None else env
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        mask = [d.strip() for d in env.get(var, "").split(",") if d.strip()]
        if mask:
            if local_rank >= len(mask):
                raise ValueError(f"local rank {local_rank} but {var}={env[var]} names {len(mask)} devices")
            if var == "ROCR_VISIBLE_DEVICES":
                return str(local_rank)         # HIP numbers the ROCR-visible devices from 0
            return mask[local_rank]
    return str(local_rank)


# ------------------------------------------------------------- per-rank host CPUs
#
# One rank keeps ~14 host cores busy per MI355X, so on a node with 8 GPUs
# the ranks must not share cores: each local rank gets a disjoint set of CPUs inside the
# NUMA node of its GPU (the ranks on one node split that node's allowed CPUs into equal
# contiguous slices), and runs cpu_share / ranks threads on it.  Everything here reads
# sysfs only: the launcher never initialises the GPU.

def cpu_quota() -> int:
    """CPUs this process may keep busy: its affinity, capped by the cgroup's CPU quota (a
    GPU box's affinity lists the whole machine but its quota grants a share)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return n


def parse_cpu_list(text: str) -> list[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11] (the kernel's cpulist format)."""
    out = []
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def format_cpu_list(cpus) -> str:
    """[0, 1, 2, 3, 8] -> '0-3,8'."""
    cpus = sorted(set(cpus))
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


def node_cpus(node: int, sysfs: str = "/sys") -> list[int]:
    try:
        with open(os.path.join(sysfs, f"devices/system/node/node{node}/cpulist")) as f:
            return parse_cpu_list(f.read())
    except OSError:
        return []


def gpu_numa_nodes(sysfs: str = "/sys") -> list[int]:
    """NUMA node of every GPU in HIP's device order (the KFD topology's GPU nodes in node
    order, as ROCr enumerates its agents), from the PCI device's numa_node; -1 where
    unknown.  [] without a KFD topology (no GPU driver, e.g. the CPU container)."""
    root = os.path.join(sysfs, "class/kfd/kfd/topology/nodes")
    try:
        ids = sorted(int(n) for n in os.listdir(root) if n.isdigit())
    except OSError:
        return []
    out = []
    for n in ids:
        props = {}
        try:
            with open(os.path.join(root, str(n), "properties")) as f:
                for ln in f:
                    k, _, v = ln.partition(" ")
                    props[k] = v.strip()
        except OSError:
            continue
        if int(props.get("simd_count", "0") or 0) == 0:
            continue                             # a CPU node
        loc, dom = int(props.get("location_id", "0")), int(props.get("domain", "0"))
        bdf = f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7:x}"
        node = -1
        try:
            with open(os.path.join(sysfs, "bus/pci/devices", bdf, "numa_node")) as f:
                node = int(f.read().strip())
        except (OSError, ValueError):
            pass
        out.append(node)
    return out


def core_keys(cpus, sysfs: str = "/sys") -> dict:
    """cpu -> its physical core's first hardware thread (SMT siblings share a key)."""
    out = {}
    for c in cpus:
        try:
            with open(os.path.join(sysfs, f"devices/system/cpu/cpu{c}/topology/thread_siblings_list")) as f:
                out[c] = min(parse_cpu_list(f.read()))
        except (OSError, ValueError):
            out[c] = c
    return out


def rank_cpu_sets(devices: list[int], allowed, gpu_nodes: list[int], node_lists: dict,
                  core_of: dict | None = None) -> tuple[list, str]:
    """Disjoint CPU sets for the local ranks whose GPUs are `devices` (HIP indices, one per
    local rank): the ranks on one NUMA node split that node's `allowed` CPUs into equal
    slices of whole physical cores (SMT siblings stay together: `core_of` maps a CPU to its
    core), in local-rank order.  A rank whose GPU's node is unknown, or whose node has fewer
    allowed CPUs than ranks on it, draws from all allowed CPUs not taken by a node split.
    Returns (per-rank sorted CPU lists, a note)."""
    core_of = core_of or {}
    allowed = sorted(set(allowed), key=lambda c: (core_of.get(c, c), c))
    nodes = [gpu_nodes[d] if 0 <= d < len(gpu_nodes) else -1 for d in devices]
    groups: dict = {}
    for r, nd in enumerate(nodes):
        groups.setdefault(nd, []).append(r)
    sets: list = [None] * len(devices)
    taken: set = set()
    notes = []
    for nd, ranks in sorted(groups.items()):
        inode = set(node_lists.get(nd, []))
        pool = [c for c in allowed if c in inode] if nd >= 0 else []
        if nd < 0 or len(pool) < len(ranks):
            continue
        share = len(pool) // len(ranks)
        for i, r in enumerate(ranks):
            sets[r] = sorted(pool[i * share:(i + 1) * share])
            taken.update(sets[r])
        notes.append(f"node{nd}: {len(ranks)} rank(s) x {share} CPUs")
    rest = [r for r in range(len(devices)) if sets[r] is None]
    if rest:
        pool = [c for c in allowed if c not in taken]
        share = len(pool) // len(rest) if pool else 0
        for i, r in enumerate(rest):
            sets[r] = sorted(pool[i * share:(i + 1) * share] if share else allowed)
        notes.append(f"no NUMA split for rank(s) {rest}: " + (f"{share} CPUs each" if share else "all allowed CPUs"))
    return sets, "; ".join(notes)


def local_cpu_sets(local_world: int, devices: list[int] | None = None) -> tuple[list, str]:
    """rank_cpu_sets for this node's local ranks (GPU k for local rank k unless `devices`
    says otherwise), over this process's affinity and the machine's sysfs."""
    devices = list(range(local_world)) if devices is None else devices
    gn = gpu_numa_nodes()
    lists = {nd: node_cpus(nd) for nd in set(gn) if nd >= 0}
    allowed = os.sched_getaffinity(0)
    return rank_cpu_sets(devices, allowed, gn, lists, core_keys(allowed))


def malloc_thp_env(env: dict | None = None) -> dict:
    """The environment for a bt2x-align (or reference aligner) child with glibc's malloc on
    transparent huge pages (GLIBC_TUNABLES glibc.malloc.hugetlb=1: malloc madvises its heaps
    MADV_HUGEPAGE, which boxes with THP in "madvise" mode need).  The aligner's per-read
    state is a few GB of small heap buffers touched in scattered order once per cohort
    pass; on 4 KiB pages nearly every context access missed the TLB.  Measured on the box
    (round 6, interleaved): 3.29 / 3.27 against 2.88 / 3.10 M reads/s, host CPU 4.46 against
    4.76-5.10 us per read.  BT2X_MALLOC_THP=0 leaves the environment as it is."""
    env = dict(os.environ if env is None else env)
    if env.get("BT2X_MALLOC_THP", "1") == "0":
        return env
    cur = env.get("GLIBC_TUNABLES", "")
    if "glibc.malloc.hugetlb" not in cur:
        env["GLIBC_TUNABLES"] = (cur + ":" if cur else "") + "glibc.malloc.hugetlb=1"
    return env


def aligner_messages(stderr: str) -> str:
    """An aligner's stderr minus its launcher-facing lines (BT2X_*) and its alignment
    summary: what a single run leaves for the user (per-read warnings)."""
    out, lines, i = [], stderr.splitlines(keepends=True), 0
    while i < len(lines):
        ln = lines[i]
        if ln.startswith("BT2X_"):
            i += 1
            continue
        if ln.rstrip("\n").endswith(" reads; of these:") or ln.rstrip("\n") == "0 reads":
            while i < len(lines) and not lines[i].rstrip("\n").endswith("overall alignment rate"):
                i += 1
            i += 1
            continue
        out.append(ln)
        i += 1
    return "".join(out)


def _split_out(args: list[str]) -> tuple[list[str], str | None]:
    args = list(args)
    for flag in ("-S", "--output"):
        if flag in args:
            i = args.index(flag)
            if i + 1 >= len(args):
                raise ValueError(f"{flag} needs a file name")
            out = args[i + 1]
            del args[i:i + 2]
            return args, out
    return args, None


def _append(dst, path: str) -> None:
    with open(path, "rb") as f:
        size = os.fstat(f.fileno()).st_size
        off = 0
        while off < size:                       # in-kernel copy; no user-space buffer pass
            n = os.sendfile(dst.fileno(), f.fileno(), off, size - off)
            if n <= 0:
                raise OSError(f"sendfile stopped at {off} of {size} bytes of {path}")
            off += n


def run_sharded(aligner: str, args: list[str], dist=None, set_device: bool = True) -> dict:
    """Run `aligner args` as this rank's shard; returns the summed metrics (every rank), the
    max of the ranks' timed-run seconds and the total reads.  Rank 0 writes the output."""
    import subprocess
    import sys
    import tempfile
    rank, world_size, local_rank = world()
    if dist is not None and dist.is_initialized():
        rank, world_size = dist.get_rank(), dist.get_world_size()
    args, out = _split_out(args)
    if out is None:                             # stdout: parts under a directory rank 0 names
        box = [tempfile.mkdtemp(prefix="bt2x_parts_") if rank == 0 else None]
        if dist is not None and dist.is_initialized() and world_size > 1:
            dist.broadcast_object_list(box, src=0)
        part_base = os.path.join(box[0], "out.sam")
    else:
        part_base = out
    part = f"{part_base}.part{rank}"
    cmd = [aligner] + args + ["-S", part, "--shard", f"{rank}/{world_size}", "--metrics"]
    if rank > 0:
        cmd.append("--no-hd")
    # this rank's own CPUs inside its GPU's NUMA node (unless the caller chose them)
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
    if local_world > 1 and "--cpus" not in args:
        sets, _ = local_cpu_sets(local_world)
        if sets[local_rank]:
            cmd += ["--cpus", format_cpu_list(sets[local_rank])]
            if "-p" not in args:
                cmd += ["-p", str(max(1, min(len(sets[local_rank]), cpu_quota() // local_world)))]
    env = malloc_thp_env()
    if set_device:
        env["HIP_VISIBLE_DEVICES"] = rank_device(local_rank, env)
    r = subprocess.run(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    res = {"rc": r.returncode, "stderr": r.stderr}
    if r.returncode == 0:
        # the per-read warnings a single run prints (printEEScoreMsg), not the launcher's
        # own lines or the shard's summary (rank 0 prints the summed one)
        sys.stderr.write(aligner_messages(r.stderr))
        sys.stderr.flush()
    try:
        got = parse_metrics(r.stderr) if r.returncode == 0 else None
    except ValueError as e:
        got, res["rc"], res["stderr"] = None, 1, r.stderr + f"\n{e}\n"
    met = got["metrics"] if got else {k: 0 for k in METRIC_NAMES}
    t_align = float(got["timed"].get("t_align", 0)) if got else 0.0
    ok = sum_counters({"failed": 1 if res["rc"] else 0}, dist)["failed"] == 0
    res["metrics"] = sum_counters(met, dist)
    res["t_align_max"] = max_over_ranks(t_align, dist)
    res["reads"] = res["metrics"]["nread"]
    res["ok"] = ok
    if ok and rank == 0:
        dst = open(out, "wb") if out else sys.stdout.buffer
        try:
            dst.flush()
            for k in range(world_size):
                _append(dst, f"{part_base}.part{k}")
            dst.flush()
        finally:
            if out:
                dst.close()
    if dist is not None and dist.is_initialized() and world_size > 1:
        dist.barrier()                           # parts are read before they go
    if ok:
        os.unlink(part)
        if out is None and rank == 0:
            os.rmdir(os.path.dirname(part_base))
    return res


def main(argv=None) -> int:
    import argparse
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    ap = argparse.ArgumentParser(prog="python -m bt2x.dist",
                                 description="bt2x-align over all ranks' GPUs, reads sharded (run under torch.distributed.run)")
    ap.add_argument("--aligner", default=os.path.join(here, "bt2x-align"))
    ap.add_argument("--no-device", action="store_true", help="do not set HIP_VISIBLE_DEVICES per rank")
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    rest = a.rest[1:] if a.rest[:1] == ["--"] else a.rest
    import torch.distributed as tdist
    use_dist = int(os.environ.get("WORLD_SIZE", "1")) > 1
    if use_dist:
        init_quiet(tdist)
    try:
        res = run_sharded(a.aligner, rest, tdist if use_dist else None, set_device=not a.no_device)
    finally:
        if use_dist:
            tdist.destroy_process_group()
    rank = world()[0]
    if res["rc"]:
        sys.stderr.write(res["stderr"])
    if rank == 0 and res["ok"]:
        sys.stderr.write(alignment_summary(res["metrics"]))
        sys.stderr.write(f"BT2X_DIST ranks={world()[1]} reads={res['reads']} t_align_max={res['t_align_max']:.4f}\n")
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    raise SystemExit(main())
