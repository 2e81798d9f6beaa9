#!/bin/bash
# Round-5 A/B on LLC-90: the correction + continuity k-march's load batch (MGCM_CORR_SB = 1: one
# level at a time, 5, 10 levels loaded before their use), alternating, then the LLC parity tests
# with batches of 5.
#   bash profiles/corr_sb.sh <out-tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for v in 1 5 10 1 5 10 1 5 10; do
  MGCM_CORR_SB=$v timeout -k 10 200 python bench.py --config llc90_synthetic --steps 40 --warmup 4 --no-cs32 \
    --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1])
k=d['kernel_ms_mean']; print('corr_sb=$v', round(d['ms_per_step'],4), k.get('cg2d'), k.get('sfp_rhs'), k.get('correction'))"
done
MGCM_CORR_SB=10 timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_llc.py \
  > $O/llc_parity.log 2>&1; tail -2 $O/llc_parity.log
