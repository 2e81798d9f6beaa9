#!/bin/bash
# (MGCM_DT_LF was an A/B-only knob, removed after these runs: all three grids long first won)
# Round 6: rocprofv3 kernel stats of the fused grids per long-first mask (MGCM_DT_LF 0 / 7 / 2),
# alternating twice on one box (dtorder2.sh's profile part).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6q}
mkdir -p $OUT
for rep in 1 2; do
for m in 0 7 2; do
  export MGCM_DT_LF=$m
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_m${m}_$rep -o run --output-format csv -- python3 bench.py --config global_ocean.90x40x15 --steps 100 --warmup 10 --no-cpu-baseline --no-cs32 > $OUT/prof_m${m}_$rep.json 2> $OUT/prof_m${m}_$rep.err || { echo prof failed; tail -5 $OUT/prof_m${m}_$rep.err; exit 1; }
  python3 - $OUT/prof_m${m}_$rep $m <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
t = 0.0
for r in csv.DictReader(open(f)):
    if "k_dt_l" in r["Name"]:
        a = float(r["AverageNs"]) / 1e3
        t += a
        print("mask", sys.argv[2], r["Name"][:30], r["Calls"], round(a, 2))
print("mask", sys.argv[2], "sum", round(t, 2))
PY
done
done
