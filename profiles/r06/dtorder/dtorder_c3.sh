#!/bin/bash
# Round 6: the long-first order on C3's k_dt_l1 (GMREDI_CALC_TENSOR | CALC_PHI_HYD beside each
# other in the staggered step): cs32x15 bench alternating default (long first) and
# MGCM_DT_LAYOUT=4 (listed order), then rocprofv3 kernel stats of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6c}
mkdir -p $OUT
for rep in 1 2 3; do
  for o in 0 4; do
    if [ $o = 0 ]; then unset MGCM_DT_LAYOUT; else export MGCM_DT_LAYOUT=$o; fi
    timeout -k 10 200 python3 bench.py --config global_ocean.cs32x15 --steps 100 --warmup 10 --no-cpu-baseline --no-cs32 > $OUT/c3_l${o}_$rep.json 2> $OUT/c3_l${o}_$rep.err || { echo bench failed; tail -5 $OUT/c3_l${o}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c3_l${o}_$rep.json')); print('C3 layout=$o', round(d['ms_per_step'],4))"
  done
done
for o in 0 4; do
  if [ $o = 0 ]; then unset MGCM_DT_LAYOUT; else export MGCM_DT_LAYOUT=$o; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_l$o -o run --output-format csv -- python3 bench.py --config global_ocean.cs32x15 --steps 100 --warmup 10 --no-cpu-baseline --no-cs32 > $OUT/prof_l$o.json 2> $OUT/prof_l$o.err || { echo prof failed; tail -5 $OUT/prof_l$o.err; exit 1; }
  python3 - $OUT/prof_l$o $o <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_dt_l" in r["Name"] or "cg2d" in r["Name"]:
        print("layout", sys.argv[2], r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
done
