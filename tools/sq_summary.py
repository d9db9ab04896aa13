#!/usr/bin/env python3
"""Summarise gpurun_out/prof_sq/run_counter_collection.csv for the bt2x kernels."""
import collections
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_sq/run_counter_collection.csv"
d = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(path)):
    k = r["Kernel_Name"]
    for tag in ("seed_kernel", "dp_fill", "dp_walk", "dp_kernel"):
        if tag in k:
            d[tag][r["Counter_Name"]] += float(r["Counter_Value"])
            d[tag]["_vgpr"] = float(r["VGPR_Count"])
for k, v in d.items():
    cyc = v.get("SQ_WAVE_CYCLES", 1)
    print(f"{k}: waves={v['SQ_WAVES']:.0f} valu_insts={v['SQ_INSTS_VALU']:.3e} vmem_rd={v['SQ_INSTS_VMEM_RD']:.3e} "
          f"active_valu/wave_cyc={v['SQ_ACTIVE_INST_VALU']/cyc:.3f} wait_any={v['SQ_WAIT_ANY']/cyc:.3f} "
          f"wait_inst={v['SQ_WAIT_INST_ANY']/cyc:.3f} active_any={v['SQ_ACTIVE_INST_ANY']/cyc:.3f}")
