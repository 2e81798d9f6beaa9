#!/bin/bash
# Iteration run on the GPU box: GPU tests (optional), then for each config a bench line
# (no CPU baseline) and a rocprofv3 kernel-stats pass.
#   TESTS=1|0  CONFIGS="global_ocean.90x40x15 llc90_synthetic"  OUT=gpurun_out/iter
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/iter}
mkdir -p $OUT
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
for c in ${CONFIGS:-global_ocean.90x40x15 llc90_synthetic}; do
  case $c in llc90_synthetic) A="--steps 48 --warmup 4";; global_ocean.cs32x15) A="--steps 100 --warmup 10";; *) A="--steps 200 --warmup 20";; esac
  timeout -k 10 300 python bench.py --config $c $A --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; tail -30 $OUT/bench_$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['ms_per_step'],4), 'ms/step', round(d['value'],2), d['unit'], {k: round(v*1e3,1) for k,v in d['kernel_ms_mean'].items()})"
  if [ "${PROF:-1}" = 1 ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 bench.py --config $c $A --no-cpu-baseline > /dev/null 2> $OUT/prof_$c.err || { echo "rocprof $c failed"; tail -20 $OUT/prof_$c.err; exit 1; }
    python - <<PY
import csv, glob
f = glob.glob("$OUT/prof_$c/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print("   %-44s %6s %9.1f us %6.2f%%" % (r["Name"].split("(")[0].replace("mgcm::", "").replace("void ", "")[:44], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
PY
  fi
done
