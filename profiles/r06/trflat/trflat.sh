#!/bin/bash
# Round 6: the tracers' whole-column march (column pairs, implicit solve inside) with its pairs
# dealt evenly over one workgroup per CU (MGCM_TRACER_MARCH2=2) against whole tile rows per
# workgroup (=1, 234 workgroups of 225 pairs on LLC-90, 22 CUs idle): parity (LLC-30 tracer
# forms, LLC-90 full size both), LLC-90 A/B alternating, then rocprofv3 kernel stats + PMC of =2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6f}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_llc.py -m gpu -x -v -s -k "tracer or full_size" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for m2 in 1 2; do
    export MGCM_TRACER_MARCH2=$m2
    timeout -k 10 200 python3 bench.py --config llc90_synthetic --steps 40 --warmup 6 --no-cpu-baseline --no-cs32 > $OUT/llc_m2${m2}_$rep.json 2> $OUT/llc_m2${m2}_$rep.err || { echo bench failed; tail -5 $OUT/llc_m2${m2}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/llc_m2${m2}_$rep.json')); print('LLC m2=$m2', round(d['ms_per_step'],4))"
  done
done
export MGCM_TRACER_MARCH2=2
MODE=prof CONFIG=llc90_synthetic TAG=${1:-r6f}/prof BENCH_ARGS="--steps 30 --warmup 4 --no-cs32" PMC_ARGS="--no-cs32" bash profiles/run_r2.sh > $OUT/prof.log 2>&1 || { echo prof failed; tail -20 $OUT/prof.log; exit 1; }
python3 - $OUT/prof <<'PY'
import csv, json, sys
o = sys.argv[1]
for r in list(csv.DictReader(open(o + "/kernel_stats.csv")))[:8]:
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
p = json.load(open(o + "/pmc_summary.json"))["kernels"]
for k, v in p.items():
    if "tracer" in k:
        print(k[:60], round(v["hbm_bytes_per_launch"] / 1e6, 1), "MB per launch")
PY
