#!/bin/bash
# Round 6: the tracer implicit solve's forward sweep inside the whole-column march
# (MGCM_TRACER_MARCH=2; measured as MGCM_TRACER_FWD=1 before the knobs were merged): LLC-30 parity + LLC-90 full-size parity with it on, LLC-90 A/B,
# a rocprofv3 kernel trace of the fused form; then the self-spawned N = 2 gloo rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6d}
mkdir -p $OUT
export TMPDIR=/tmp
MGCM_TRACER_MARCH=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_llc.py -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_fwd.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error" $OUT/pytest_fwd.log | head; tail -30 $OUT/pytest_fwd.log; exit 1; }
tail -1 $OUT/pytest_fwd.log
for rep in 1 2; do
  for fw in 0 1; do
    MGCM_TRACER_MARCH=$((fw + 1)) timeout -k 10 200 python3 bench.py --config llc90_synthetic --steps 40 --warmup 10 --no-cpu-baseline > $OUT/llc_fwd${fw}_$rep.json 2> $OUT/llc_fwd${fw}_$rep.err || { echo bench llc failed; tail -5 $OUT/llc_fwd${fw}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/llc_fwd${fw}_$rep.json')); k=d['kernel_ms_mean']; print('LLC fwd=$fw', round(d['ms_per_step'],4), 'temp_step ms', round(k['temp_step'],4), 'cg2d', round(k['cg2d'],4))"
  done
done
MGCM_TRACER_MARCH=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_fwd -o run -- python3 bench.py --config llc90_synthetic --steps 40 --warmup 10 --no-cpu-baseline > $OUT/prof_fwd.log 2>&1 || { echo rocprof failed; tail -5 $OUT/prof_fwd.log; exit 1; }
find $OUT/prof_fwd -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-4 {} | head -14'
MGCM_SHARD_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_n2.json 2> $OUT/bench_n2.err || { echo bench n2 failed; tail -5 $OUT/bench_n2.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_n2.json')); print('N2', d['n_gpus'], d['distinct_gpus'], round(d['value'],1), [(r['config'], r.get('ms_per_step'), r.get('error')) for r in d.get('sharded', [])])"
