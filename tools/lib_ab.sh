#!/bin/bash
# A/B of diagnostic library builds (LIBS="name:path ...", "default" = the in-tree library) on
# CONFIGS, alternating.   OUT=gpurun_out/libab
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${OUT:-gpurun_out/libab}
mkdir -p $OUT
for r in 1 2; do
  for c in ${CONFIGS:-llc90_synthetic}; do
    st=400; [ $c = global_ocean.cs32x15 ] && st=200; [ $c = llc90_synthetic ] && st=30
    for v in ${LIBS:-default}; do
      n=${v%%:*}; lib=${v#*:}; [ $n = default ] && lib=mitgcm_amd/libmitgcm_amd.so
      MGCM_LIB=$PWD/$lib timeout -k 10 200 python bench.py --config $c --steps $st --warmup 10 --no-cpu-baseline > $OUT/b_${n}_${c}_$r.json 2> $OUT/e_${n}_${c}_$r.err || { echo "bench $n $c failed"; tail -5 $OUT/e_${n}_${c}_$r.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/b_${n}_${c}_$r.json')); print('$c', '$n', $r, round(d['ms_per_step'],4))"
    done
  done
done
