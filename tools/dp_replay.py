#!/usr/bin/env python3
"""DP-kernel A/B on the GPU (development tool).

Records the DP launches bt2x-align makes for one FASTQ file of simulated 150 bp reads
(bench.py's genome/read generators and index builder, a smaller genome by default: DP
shapes depend on the reads, --dpad and the in-flight count, not on the genome size), then
replays only those launches from HBM under each configuration given as an environment
assignment list, e.g.

    python tools/dp_replay.py --slots 1048576 "" BT2X_DP_ABLATE=1 BT2X_DP_ABLATE=2

prints per configuration the DP milliseconds per replay step (HIP events on the launch
stream, mean of --steps) and the kernel counters.
"""
from __future__ import annotations

import argparse
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omp-bowtie2-prime_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genome-mb", type=float, default=400.0)
    ap.add_argument("--reads", type=int, default=1 << 20)
    ap.add_argument("--slots", type=int, default=65536, help="reads in flight while recording")
    ap.add_argument("--dpad", type=int, default=12)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--workdir", default=f"/tmp/bt2x_dprep_{os.getuid()}")
    ap.add_argument("configs", nargs="*", default=[""])
    args = ap.parse_args()
    import numpy as np
    import bench

    ns = argparse.Namespace(genome_mb=args.genome_mb, genome_seed=2024, reads=args.reads, steps=1, warmup=0,
                            read_len=150, replay_reads=args.reads, dpad=args.dpad, no_legs=True)
    os.makedirs(args.workdir, exist_ok=True)
    chroms, codes, warm, steps, per = bench.make_inputs(ns, 0, 1, args.workdir)
    base, _ = bench.build_index(ns, chroms, codes, args.workdir, 0, None)
    del chroms, codes
    fq = steps[0]
    ddir = os.path.join(args.workdir, f"dump_{args.slots}")
    if not os.path.exists(os.path.join(ddir, "done")):
        shutil.rmtree(ddir, ignore_errors=True)
        os.makedirs(ddir)
        rargs = argparse.Namespace(rss_limit_gb=200.0)
        bench.run_aligner(rargs, [bench.ALIGN, "-x", base, "-U", fq, "-S", os.devnull, "--dpad", str(args.dpad), "-p",
                                  str(bench.cpu_share()), "--slots", str(args.slots), "--dump", ddir, "--no-pipeline"],
                          os.path.join(args.workdir, "dump.err"), "launch recording")
        open(os.path.join(ddir, "done"), "w").close()
    launches = [(k, p) for k, p in bench.load_dumps(ddir) if k == "dp"]
    import torch
    from bt2x import abi, lib
    dev = torch.device("cuda", 0)
    ctx = lib.Context(lib.Index(base, load_offs=True), device=0)

    def to_dev(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)

    plan = []
    for _, parts in launches:
        m = len(parts[3])
        rec_cap, edit_cap = int(parts[4][0]) + 1024, int(parts[4][1]) + 4096
        fl = parts[3]["flags"]
        lf = (abi.DPL_I16 if (fl & abi.DP_I16).any() else 0) | (abi.DPL_REF_TEXT if (fl & abi.DP_REF_TEXT).any() else 0)
        refs = parts[2] if len(parts[2]) else np.zeros(1, dtype=np.uint8)
        plan.append((m, [to_dev(parts[0]), to_dev(parts[1]), to_dev(refs), to_dev(parts[3]),
                         torch.empty(m * abi.DP_OUT.itemsize, dtype=torch.uint8, device=dev),
                         torch.empty(rec_cap * abi.ALN_REC.itemsize, dtype=torch.uint8, device=dev),
                         torch.empty(edit_cap * 4, dtype=torch.uint8, device=dev),
                         torch.zeros(16, dtype=torch.int32, device=dev), rec_cap, edit_cap, lf]))
    del launches
    sh = torch.cuda.current_stream(dev).cuda_stream
    nprob = sum(m for m, _ in plan)
    print(f"# {len(plan)} DP launches, {nprob} problems (recorded at --slots {args.slots})", flush=True)

    def step(counters=None):
        ms = 0.0
        for m, b in plan:
            ctx.dp_align_dev(b[0].data_ptr(), b[1].data_ptr(), b[2].data_ptr(), b[3].data_ptr(), m,
                             b[4].data_ptr(), b[5].data_ptr(), b[8], b[6].data_ptr(), b[9],
                             b[7].data_ptr(), sh, launch_flags=b[10])
            ms += ctx.last_kernel_ms(abi.K_DP)
            if counters is not None:
                for k, v in ctx.last_counters(abi.K_DP).items():
                    counters[k] = counters.get(k, 0) + v
        return ms

    for cfg in args.configs:
        cfg = cfg.strip('"\'')                        # "" from a shell word: the default
        env = dict(kv.split("=", 1) for kv in cfg.split(",") if kv)
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        ctr = {}
        step(ctr)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        mss = [step() for _ in range(args.steps)]
        torch.cuda.synchronize(dev)
        wall = (time.perf_counter() - t0) / args.steps
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        print(f"config [{cfg or 'default'}]: DP {np.mean(mss):.2f} ms/step (min {min(mss):.2f}), wall {wall * 1e3:.1f} ms; "
              f"bt_cells {ctr.get('bt_cells', 0)} computed {ctr.get('dp_cells_computed', 0)}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
