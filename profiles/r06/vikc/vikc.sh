#!/bin/bash
# Round 6: k_mom_vi_m2's levels per workgroup on LLC-90 (MGCM_VI_KC, an A/B-only override):
# 25 (two chunks, 936 workgroups = 1.83 rounds of 512 resident at 2 per CU) against 50 (one
# chunk, 468 workgroups, one round) and 17 (three chunks); alternating, bench lines + the
# eager pass's per-kernel means.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6k}
mkdir -p $OUT
for rep in 1 2; do
  for kc in 25 50 17; do
    MGCM_VI_KC=$kc timeout -k 10 200 python3 bench.py --config llc90_synthetic --steps 40 --warmup 6 --no-cpu-baseline --no-cs32 > $OUT/llc_kc${kc}_$rep.json 2> $OUT/llc_kc${kc}_$rep.err || { echo bench failed; tail -5 $OUT/llc_kc${kc}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/llc_kc${kc}_$rep.json')); print('LLC kc=$kc', round(d['ms_per_step'],4), 'mom', round(d['kernel_ms_mean']['mom_step']*1e3,1))"
  done
done
