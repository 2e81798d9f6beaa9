#!/bin/bash
# Round 6: the tracers' whole-column march with the implicit solve one column per thread
# (MGCM_TRACER_MARCH=4) against the column-pair form (=3, the default): parity (LLC-30 every
# form, LLC-90 full size both), LLC-90 A/B alternating, then rocprofv3 kernel stats + PMC of =4.
# (=4 was slower -- 269 against 216 us per tracer -- and was removed after this run)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6t}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_llc.py -m gpu -x -v -s --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for tm in 3 4; do
    if [ $tm = 0 ]; then unset MGCM_TRACER_MARCH; else export MGCM_TRACER_MARCH=$tm; fi
    timeout -k 10 200 python3 bench.py --config llc90_synthetic --steps 40 --warmup 6 --no-cpu-baseline --no-cs32 > $OUT/llc_tm${tm}_$rep.json 2> $OUT/llc_tm${tm}_$rep.err || { echo bench failed; tail -5 $OUT/llc_tm${tm}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/llc_tm${tm}_$rep.json')); k=d['kernel_ms_mean']; print('LLC tm=$tm', round(d['ms_per_step'],4), {a: round(b,4) for a, b in k.items() if 'tr' in a or 'thermo' in a})"
  done
done
export MGCM_TRACER_MARCH=4
MODE=prof CONFIG=llc90_synthetic TAG=${1:-r6t}/prof4 BENCH_ARGS="--steps 30 --warmup 4 --no-cs32" PMC_ARGS="--no-cs32" bash profiles/run_r2.sh > $OUT/prof4.log 2>&1 || { echo prof failed; tail -20 $OUT/prof4.log; exit 1; }
python3 - $OUT/prof4 <<'PY'
import csv, json, sys
o = sys.argv[1]
for r in list(csv.DictReader(open(o + "/kernel_stats.csv")))[:8]:
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
p = json.load(open(o + "/pmc_summary.json"))["kernels"]
for k, v in p.items():
    if "tracer" in k:
        print(k[:60], round(v["hbm_bytes_per_launch"] / 1e6, 1), "MB per launch")
PY
