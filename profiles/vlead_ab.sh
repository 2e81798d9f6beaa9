#!/bin/bash
# Round-5 A/B on LLC-90: the velocities' blocking exchange at the next step's start beside
# DO_OCEANIC_PHYS (MG_FUSE_VLEAD, with the tracers' exchange on their stream, MG_FUSE_TREX: the
# new default) against the round-4 default mask (3469) and TREX alone (3533), alternating;
# then the LLC parity tests with the default.
#   bash profiles/vlead_ab.sh <out-tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for v in new 3469 3533 new 3469 3533 new 3469 3533; do
  if [ $v = new ]; then unset MGCM_STEP_FUSE; else export MGCM_STEP_FUSE=$v; fi
  timeout -k 10 200 python bench.py --config llc90_synthetic --steps 40 --warmup 4 --no-cs32 \
    --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1])
k=d['kernel_ms_mean']; print('fuse=$v', round(d['ms_per_step'],4), k.get('cg2d'), k.get('exchange'))"
done
unset MGCM_STEP_FUSE
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_llc.py \
  > $O/llc_parity.log 2>&1; tail -2 $O/llc_parity.log
