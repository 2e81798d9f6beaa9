#!/bin/bash
# (MGCM_DT_LF was an A/B-only knob, removed after these runs: all three grids long first won)
# Round 6: the fused grids' long-first order per grid (MGCM_DT_LF, A/B only: bit g-1 = grid g
# long first; 0 = the listed order everywhere, 7 = all three long first, 2 = k_dt_l2 only):
# C2 bench alternating, then rocprofv3 kernel stats of each mask on the same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6p}
mkdir -p $OUT
MGCM_DT_LF=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_ocean90.py -m gpu -x -q -k "10_steps and None" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for m in 0 7 2; do
    MGCM_DT_LF=$m timeout -k 10 200 python3 bench.py --config global_ocean.90x40x15 --steps 200 --warmup 20 --no-cpu-baseline --no-cs32 > $OUT/c2_m${m}_$rep.json 2> $OUT/c2_m${m}_$rep.err || { echo bench failed; tail -5 $OUT/c2_m${m}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c2_m${m}_$rep.json')); print('C2 mask=$m', round(d['ms_per_step'],4), round(d['kernel_ms_mean']['mom_step']*1e3,1))"
  done
done
for m in 0 7 2; do
  export MGCM_DT_LF=$m
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_m$m -o run --output-format csv -- python3 bench.py --config global_ocean.90x40x15 --steps 100 --warmup 10 --no-cpu-baseline --no-cs32 > $OUT/prof_m$m.log 2>&1 || { echo prof failed; tail -5 $OUT/prof_m$m.log; exit 1; }
  python3 - $OUT/prof_m$m $m <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_dt_l" in r["Name"] or "cg2d_bxy" in r["Name"]:
        print("mask", sys.argv[2], r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
done
