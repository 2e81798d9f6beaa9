#!/bin/bash
# Round-5 A/B of the single-CU CG2D's barrier-lifted iteration (MGCM_CG2D_LB = 0..3, the
# bit-0 / bit-1 re-derived neighbours of kernels_solve.hip k_cg2d_bxy): C2 bench per variant,
# then the 10-step device-order-oracle parity at the lifted variants.
#   bash profiles/cg_lb.sh <out-tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for lb in 0 1 2 3 0; do
  MGCM_CG2D_LB=$lb timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cs32 --no-cpu-baseline \
    > $O/bench_lb$lb.json 2> $O/bench_lb$lb.err || { tail -20 $O/bench_lb$lb.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_lb$lb.json').read().strip().splitlines()[-1])
print('LB=$lb', round(d['ms_per_step'],4), 'us/it', round(d['roofline']['us_per_iteration'],4))"
done
for lb in 1 2 3; do
  MGCM_CG2D_LB=$lb timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
    tests/test_gpu_ocean90.py -k "10_steps" > $O/parity_lb$lb.log 2>&1 || { tail -20 $O/parity_lb$lb.log; exit 1; }
  tail -1 $O/parity_lb$lb.log
done
