"""Debug: lane-kernel i16 candidate mismatches in slow-path waves."""
import os, sys
sys.path.insert(0, "tests"); sys.path.insert(0, "omp-bowtie2-prime_amd"); sys.path.insert(0, "tools")
os.environ["BT2X_DP_WAVE"] = "0"
import numpy as np
import golden_io as g, oracle_lib as ol
from bt2x import abi, lib
import test_gpu_parity as t
base = g.materialize_index("rep", "/tmp/dbgidx")
ctx = lib.Context(lib.Index(base, load_offs=True))
rd, qu, rf, inp = t._random_dp_problems(6000, seed=77 + 10, i16=1.0)
grp = inp[640:704].copy()
def run(sel, label):
    out, recs, edits, dig, cands = ctx.dp_align(rd, qu, rf, sel, debug=True)
    eo, erecs, eedits, edig, ecands, _ = ol.dp_align(ol.default_scoring(), rd, qu, rf, sel)
    cb = np.nonzero((cands != ecands).any(axis=1))[0]
    bb = np.nonzero(out["best"] != eo["best"])[0]
    db = np.nonzero((dig != edig).any(axis=1))[0]
    print(label, "n", len(sel), "cand bad", len(cb), "best bad", len(bb), "dig bad", len(db), "minsc min", sel["minsc"].min())
    for i in cb[:3]:
        print("  lane", i, "R", sel[i]["rdlen"], "C", sel[i]["ncol"], "minsc", sel[i]["minsc"], "best", out["best"][i], eo["best"][i],
              "ncand", out["ncand"][i], eo["ncand"][i])
        print("   ours", [abi.cand_fields(c, True)[1:] for c in cands[i][:6]])
        print("   exp ", [abi.cand_fields(c, True)[1:] for c in ecands[i][:6]])
run(grp, "wave10")
m = grp["minsc"] >= -254
run(grp[m], "wave10 minsc>=-254 only")
for lo in (-260, -300, -400, -600):
    g2 = grp.copy(); g2["minsc"] = np.maximum(g2["minsc"], lo); run(g2, f"clamped to {lo}")
g3 = grp.copy(); g3["rdlen"] = np.minimum(g3["rdlen"], 40); run(g3, "R<=40")
g4 = grp.copy(); g4["ncol"] = np.minimum(g4["ncol"], 60); run(g4, "C<=60")
