#!/bin/bash
# round 5: the small-launch DP threshold (BT2X_DP_WAVE_MAX: launches up to it run one wave
# per problem, unbanded) -- the timed C3 run under rocprofv3 kernel stats, per setting
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-r05o}
for wm in ${WMS:-32768 8192 2048}; do
	BT2X_DP_WAVE_MAX=$wm timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_wm$wm -o run -- \
		python3 bench.py --steps 20 --warmup 5 --runs 1 --no-cpu --no-legs --no-rep-leg --no-replay > gpurun_out/${TAG}_wm$wm.json 2> gpurun_out/${TAG}_wm$wm.err
	rc=$?; echo "wave_max=$wm rc=$rc"; [ $rc -eq 0 ] || exit $rc
	python3 - "$TAG" "$wm" <<'PY'
import csv, glob, json, sys
tag, wm = sys.argv[1], sys.argv[2]
d = json.load(open(f"gpurun_out/{tag}_wm{wm}.json"))
f = glob.glob(f"gpurun_out/{tag}_wm{wm}/**/*kernel_stats.csv", recursive=True)
tot = {}
for r in csv.DictReader(open(f[0])):
    n = r["Name"]
    k = "dp_fill" if "dp_fill" in n else "dp_duo" if "dp_duo" in n else "wave<0" if "dp_wave_kernel<0" in n else \
        "wave<1>" if "dp_wave_kernel<1" in n else "wave<2>" if "dp_wave_kernel<2" in n else None
    if k: tot[k] = tot.get(k, 0) + float(r["TotalDurationNs"]) * 1e-6
g = d.get("end_to_end", {}).get("gpu", {})
print(f"wave_max={wm}: value={d['value']} k_dp={g.get('k_dp')} ms:", {k: round(v, 1) for k, v in tot.items()})
PY
done
