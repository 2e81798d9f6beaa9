#!/bin/bash
# Round 6 A/B: the staggered cube's two launch folds (MG_FUSE_RINGP: the halo-ring AB2 in
# DO_OCEANIC_PHYS's grid, k_phys_ring; MG_FUSE_ENDS: DO_STAGGER_FIELDS_EXCHANGES' u, v, w in
# CALC_R_STAR's grid, k_rstar_exmix) against the round-5 launch set (MGCM_STEP_FUSE=3469).
# Parity first (the cube's GPU tests, default mask), then alternating bench runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6x}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_cs32x15.py tests/test_gpu_advect_cs.py tests/test_gpu_llc.py tests/test_gpu_refhost.py -m gpu -x -v -s --timeout 200 --timeout-method thread > $OUT/pytest_ab.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error" $OUT/pytest_ab.log | head; tail -30 $OUT/pytest_ab.log; exit 1; }
tail -1 $OUT/pytest_ab.log
for rep in 1 2 3; do
  for mask in 3469 15757; do
    MGCM_STEP_FUSE=$mask timeout -k 10 200 python3 bench.py --config global_ocean.cs32x15 --steps 200 --warmup 20 --no-cpu-baseline > $OUT/c3_m${mask}_$rep.json 2> $OUT/c3_m${mask}_$rep.err || { echo bench failed; tail -5 $OUT/c3_m${mask}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c3_m${mask}_$rep.json')); print('C3 mask=$mask', round(d['ms_per_step'],4), round(d['cg2d_mean_iters_per_solve'],1))"
  done
done
