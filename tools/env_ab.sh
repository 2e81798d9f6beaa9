#!/bin/bash
# A/B of environment settings (ARMS="name:VAR=val,VAR2=val ..."; "base:" = none) on CONFIG,
# alternating.   OUT=gpurun_out/envab
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${OUT:-gpurun_out/envab}
CONFIG=${CONFIG:-llc90_synthetic}
st=400; [ $CONFIG = global_ocean.cs32x15 ] && st=200; [ $CONFIG = llc90_synthetic ] && st=30
mkdir -p $OUT
for r in 1 2; do
  for a in ${ARMS:-base:}; do
    n=${a%%:*}; e=${a#*:}
    env ${e//,/ } timeout -k 10 200 python bench.py --config $CONFIG --steps $st --warmup 10 --no-cpu-baseline > $OUT/b_${n}_$r.json 2> $OUT/e_${n}_$r.err || { echo "bench $n failed"; tail -5 $OUT/e_${n}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_${n}_$r.json')); print('$CONFIG', '$n', $r, round(d['ms_per_step'],4))"
  done
done
