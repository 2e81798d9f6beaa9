#!/bin/bash
# (historical: k_tr_rhs_both / MGCM_TR_BOTH were removed after this A/B -- slower)
# Round 6: the staggered cube's tracer right-hand side with both tracers of a point per thread
# (k_tr_rhs_both, shared operands loaded once; MGCM_TR_BOTH=1) against one tracer per thread
# (k_tr_rhs_pair; =0). Parity first (tests over every path of the tracer body), then C3
# alternating, then the kernels' rocprof times.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6tb}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_cs32x15.py tests/test_gpu_3d.py tests/test_gpu_options.py tests/test_gpu_advect_cs.py -m gpu -x -v -s --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
MGCM_TR_BOTH=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_cs32x15.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_pair.log 2>&1 || { echo pytest pair failed; tail -30 $OUT/pytest_pair.log; exit 1; }
tail -1 $OUT/pytest_pair.log
for rep in 1 2 3; do
  for b in 0 1; do
    MGCM_TR_BOTH=$b timeout -k 10 200 python3 bench.py --config global_ocean.cs32x15 --steps 200 --warmup 20 --no-cpu-baseline > $OUT/c3_b${b}_$rep.json 2> $OUT/c3_b${b}_$rep.err || { echo bench failed; tail -5 $OUT/c3_b${b}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c3_b${b}_$rep.json')); print('C3 both=$b', round(d['ms_per_step'],4))"
  done
done
for b in 0 1; do
  MGCM_TR_BOTH=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof$b -o run --output-format csv -- python3 bench.py --config global_ocean.cs32x15 --steps 100 --warmup 10 --no-cpu-baseline > $OUT/prof$b.json 2> $OUT/prof$b.err || { echo rocprof failed; tail -5 $OUT/prof$b.err; exit 1; }
  f=$(find $OUT/prof$b -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'tr_rhs' in r['Name'] or 'cg2d' in r['Name']: print('both=$b', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')"
done
