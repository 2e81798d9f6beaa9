#!/bin/bash
# A/B of the scheduler-strategy builds (tools/sched_variant.sh) against the default library on
# configs 2, 3 and 5, alternating.   OUT=gpurun_out/schedab
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=${OUT:-gpurun_out/schedab}
mkdir -p $OUT
D=mitgcm_amd/_build/diag
for r in 1 2; do
  for c in global_ocean.90x40x15 global_ocean.cs32x15 llc90_synthetic; do
    st=400; [ $c = global_ocean.cs32x15 ] && st=200; [ $c = llc90_synthetic ] && st=30
    for v in default max-ilp max-memory-clause; do
      lib=mitgcm_amd/libmitgcm_amd.so; [ $v != default ] && lib=$D/libmitgcm_amd_sched_$v.so
      MGCM_LIB=$PWD/$lib timeout -k 10 200 python bench.py --config $c --steps $st --warmup 10 --no-cpu-baseline > $OUT/b_${v}_${c}_$r.json 2> $OUT/e_${v}_${c}_$r.err || { echo "bench $v $c failed"; tail -5 $OUT/e_${v}_${c}_$r.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/b_${v}_${c}_$r.json')); print('$c', '$v', $r, round(d['ms_per_step'],4))"
    done
  done
done
