#!/bin/bash
# MGCM_STEP_FUSE masks A/B on one box, alternating: CONFIGS x MASKS bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/fuseab}
mkdir -p $OUT
for rep in 1 2; do
for c in ${CONFIGS:-global_ocean.90x40x15 global_ocean.cs32x15}; do
  for mk in ${MASKS:-13 45}; do
    st=300; [ $c = llc90_synthetic ] && st=24
    MGCM_STEP_FUSE=$mk timeout -k 10 200 python bench.py --config $c --steps $st --warmup 20 --no-cpu-baseline > $OUT/b_${c}_$mk.json 2> $OUT/e_${c}_$mk.err || { echo "bench $c $mk failed"; tail -20 $OUT/e_${c}_$mk.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b_${c}_$mk.json')); print('$rep $c mask $mk', 'ms/step %.4f' % d['ms_per_step'])"
  done
done
done
