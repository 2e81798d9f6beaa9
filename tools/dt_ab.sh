#!/bin/bash
# A/B of config 2's step with THERMODYNAMICS folded into DYNAMICS' launches (default) against
# the second-stream fork (MGCM_STEP_FUSE=13), alternating on one box.   OUT=gpurun_out/dtab
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${OUT:-gpurun_out/dtab}
CONFIG=${CONFIG:-global_ocean.90x40x15}
mkdir -p $OUT
for r in 1 2 3; do
  for arm in ${ARMS:-dt:141 fork:13}; do
    n=${arm%%:*}; mask=${arm##*:}
    MGCM_STEP_FUSE=$mask MGCM_OVERLAP=1 timeout -k 10 120 python bench.py --config $CONFIG --steps 400 --warmup 40 --no-cpu-baseline > $OUT/b_${n}_$r.json 2> $OUT/e_${n}_$r.err || { echo "bench $n failed"; tail -5 $OUT/e_${n}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${n}_$r.json')); print('$n', $r, round(d['ms_per_step'],4))"
  done
done
