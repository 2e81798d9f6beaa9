#!/bin/bash
# LLC-90 step against MGCM_TR_LDSPAD (unused LDS per tracer workgroup: fewer tracer
# workgroups per CU beside the pressure solve), alternating.   OUT=gpurun_out/trpad
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${OUT:-gpurun_out/trpad}
CONFIG=${CONFIG:-llc90_synthetic}
mkdir -p $OUT
for r in 1 2; do
  for pad in ${PADS:-0 41000 54000 81000}; do
    MGCM_TR_LDSPAD=$pad timeout -k 10 200 python bench.py --config $CONFIG --steps 30 --warmup 6 --no-cpu-baseline > $OUT/b_${pad}_$r.json 2> $OUT/e_${pad}_$r.err || { echo "bench $pad failed"; tail -5 $OUT/e_${pad}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${pad}_$r.json')); print('pad', $pad, $r, round(d['ms_per_step'],4))"
  done
done
