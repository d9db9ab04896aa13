#!/usr/bin/env python3
"""Turn rocprofv3 output of tools/profile_e2e.sh into committed profile summaries.

Inputs (a gpurun_out/ tree): prof_kt/run_kernel_stats.csv (+ run_kernel_trace.csv),
prof_fetch/run_counter_collection.csv (--pmc FETCH_SIZE), prof_write/... (WRITE_SIZE).
Outputs under profiles/: <tag>_kernel_stats.csv (verbatim), <tag>_bt2x_trace.csv (our
kernels' dispatches), <tag>_pmc.csv (our kernels' counter rows) and <tag>_traffic.json:
per-launch HBM traffic per kernel, corrected as MI355X_MICROARCH.md prescribes for
gfx950 (FETCH_SIZE, reported in KiB, counts half the bytes of wide reads -> x2;
WRITE_SIZE in KiB taken as is).  bench.py reads <tag>_traffic.json for
roofline.traffic when the workload key matches its own run.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import shutil
from collections import defaultdict

# logical op -> the kernels one call launches (per-launch figures are summed over them)
KERNELS = {"seed": ("seed_init_kernel", "seed_kernel"), "resolve": ("sa_resolve_kernel",),
           "round": ("round_prep_kernel", "round_sample_kernel"),
           "dp": ("dp_fill_kernel", "dp_duo_kernel", "dp_walk_kernel", "dp_wave_kernel", "dp_kernel")}


def short(name: str) -> str | None:
    for k, pats in KERNELS.items():
        for pat in pats:
            if pat in name:
                return k
    return None


def kname(name: str) -> str:
    """Kernel identity within a logical op (template arguments and namespaces dropped)."""
    base = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return base.split("(")[0].split("<")[0].strip()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default="gpurun_out")
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--workload", required=True, help="bench.py workload key of the profiled run")
    ap.add_argument("--cmd", default="python3 bench.py --no-cpu")
    ap.add_argument("--replays", type=int, default=0,
                    help="bench steps in the profiled run (warmup + steps): traffic is then reported per step "
                         "(all launches of the op in one replay), as bench.py times it")
    ap.add_argument("--segment", type=int, default=-1,
                    help="with legs on: keep only the K-th replay of bench.py's process (0: C3, 1: the C2 leg, "
                         "2: the repeat-heavy leg), the replays being the dispatch runs separated by gaps of "
                         "more than --gap-s seconds (the legs' aligner runs)")
    ap.add_argument("--gap-s", type=float, default=2.0)
    ap.add_argument("--out", default="", help="output directory (default: the repo's profiles/)")
    a = ap.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = a.out or os.path.join(root, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(a.src, "prof_kt", "run_kernel_stats.csv"),
                os.path.join(out, f"{a.tag}_kernel_stats.csv"))
    def replay_rows(path):
        """Rows of bench.py's own process, i.e. the kernel replay: of the processes that ran
        our kernels (bench.py, and the bt2x-align runs it starts as children, which finish
        first) the one whose first dispatch came last."""
        with open(path) as f:
            rows = [r for r in csv.DictReader(f) if short(r["Kernel_Name"])]
        # (rocprofv3 writes one table for all processes; without a process column the
        # issuing thread tells them apart)
        pid = next((k for k in ("Process_Id", "Thread_Id") if rows and k in rows[0]), None)
        if pid:
            first = {}
            for r in rows:
                t = int(r.get("Start_Timestamp") or r.get("Start_Time") or 0)
                first[r[pid]] = min(first.get(r[pid], t), t)
            keep = max(first, key=first.get)
            if a.segment >= 0:
                # legs on: the aligner runs of the legs start after bench.py's first replay; bench.py
                # is their parent, so the lowest process id
                keep = min(first, key=lambda k: int(k))
            rows = [r for r in rows if r[pid] == keep]
        if a.segment >= 0 and rows:
            def ts(r):
                return int(r.get("Start_Timestamp") or r.get("Start_Time") or 0)
            rows.sort(key=ts)
            seg, last = [[]], None
            for r in rows:
                if last is not None and ts(r) - last > a.gap_s * 1e9:
                    seg.append([])
                seg[-1].append(r)
                last = ts(r)
            rows = seg[a.segment] if a.segment < len(seg) else []
        return rows

    dur = defaultdict(lambda: defaultdict(list))
    with open(os.path.join(a.src, "prof_kt", "run_kernel_trace.csv")) as f, \
            open(os.path.join(out, f"{a.tag}_bt2x_trace.csv"), "w", newline="") as g:
        rd = csv.DictReader(f)
        wr = csv.DictWriter(g, fieldnames=rd.fieldnames)
        wr.writeheader()
        for r in replay_rows(os.path.join(a.src, "prof_kt", "run_kernel_trace.csv")):
            k = short(r["Kernel_Name"])
            wr.writerow(r)
            dur[k][kname(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    ctr = defaultdict(lambda: defaultdict(lambda: defaultdict(list)))
    rows = []
    for sub in ("prof_fetch", "prof_write"):
        for r in replay_rows(os.path.join(a.src, sub, "run_counter_collection.csv")):
            k = short(r["Kernel_Name"])
            rows.append(r)
            ctr[k][r["Counter_Name"]][kname(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    if rows:
        with open(os.path.join(out, f"{a.tag}_pmc.csv"), "w", newline="") as g:
            wr = csv.DictWriter(g, fieldnames=list(rows[0].keys()))
            wr.writeheader()
            wr.writerows(rows)
    res = {"workload": a.workload, "command": a.cmd,
           "correction": "traffic = 2 x FETCH_SIZE(KiB) x 1024 + WRITE_SIZE(KiB) x 1024 per launch "
                         "(gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md HBM section); Infinity-Cache "
                         "hits are included by the counters; per-call figures sum the op's kernels",
           "kernels": {}}

    def per_call(d):            # mean per launch of each kernel, summed over the op's kernels
        return sum(sum(v) / len(v) for v in d.values() if v)

    for k in KERNELS:
        f = ctr[k].get("FETCH_SIZE", {})
        w = ctr[k].get("WRITE_SIZE", {})
        if not f or not w:
            continue
        if a.replays:           # per step: every dispatch of the op over the replays
            fetch = sum(sum(v) for v in f.values()) * 1024 * 2 / a.replays
            write = sum(sum(v) for v in w.values()) * 1024 / a.replays
        else:
            fetch = per_call(f) * 1024 * 2
            write = per_call(w) * 1024
        res["kernels"][k] = {"fetch_bytes": round(fetch), "write_bytes": round(write),
                             "traffic_bytes": round(fetch + write),
                             "kernels": sorted(set(f) | set(w)),
                             "per": "step" if a.replays else "launch",
                             "avg_duration_ms": round(per_call(dur[k]) / 1e6, 4) if dur.get(k) else None,
                             "per_kernel_ms": {n: round(sum(v) / len(v) / 1e6, 4) for n, v in dur[k].items()}}
    # SQ counters (prof_sq): per step of the replay, per DP kernel; VALU utilisation =
    # VALU instructions / (kernel time x issue peak: 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles
    # per wave64 VALU op), SQ_WAIT_ANY per wave-cycle (MI355X_MICROARCH.md PMC section)
    sq_path = os.path.join(a.src, "prof_sq", "run_counter_collection.csv")
    if os.path.exists(sq_path) and a.replays:
        sq = defaultdict(lambda: defaultdict(float))
        for r in replay_rows(sq_path):
            sq[kname(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
        issue_peak = 256 * 4 * 2.4e9 / 2
        out_sq = {"what": "SQ counters of the DP kernels per bench replay step (tools/gpujobs/profile_r03.sh, "
                          "rocprofv3 --pmc); time per step from the kernel trace",
                  "workload": a.workload, "kernels": {}}
        for kn, c in sq.items():
            if "dp_" not in kn:
                continue
            c = {k: v / a.replays for k, v in c.items()}
            t = sum(sum(v) for n, v in dur["dp"].items() if n == kn) / 1e9 / a.replays if dur.get("dp") else 0
            e = dict(c)
            if c.get("SQ_WAVE_CYCLES"):
                e["wait_any_per_wave_cycle"] = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]
                e["active_per_wave_cycle"] = c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
            if t:
                e["time_s_per_step"] = t
                e["valu_util"] = c.get("SQ_INSTS_VALU", 0) / (t * issue_peak)
            out_sq["kernels"][kn] = e
        with open(os.path.join(out, f"{a.tag}_dp_sq.json"), "w") as g:
            json.dump(out_sq, g, indent=1)
        fill = out_sq["kernels"].get("dp_fill_kernel", {})
        if "dp" in res["kernels"] and fill:
            res["kernels"]["dp"]["valu_util"] = round(fill.get("valu_util", 0), 4)
            res["kernels"]["dp"]["sq_wait_any_per_wave_cycle"] = round(fill.get("wait_any_per_wave_cycle", 0), 4)
            res["kernels"]["dp"]["sq_src"] = f"profiles/{a.tag}_dp_sq.json"
    with open(os.path.join(out, f"{a.tag}_traffic.json"), "w") as g:
        json.dump(res, g, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
