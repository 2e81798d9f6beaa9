#!/bin/bash
# DO_OCEANIC_PHYS + CALC_PHI_HYD fused column pass (MG_FUSE_PHYS, MGCM_PHYS_NC columns per
# workgroup) against the two launches (MGCM_STEP_FUSE=13), LLC-90 bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/phys}
mkdir -p $OUT
for arm in ${ARMS:-off nc16 nc32 nc64}; do
  case $arm in off) E="MGCM_STEP_FUSE=13";; nc*) E="MGCM_STEP_FUSE=29 MGCM_PHYS_NC=${arm#nc}";; esac
  env $E timeout -k 10 200 python bench.py --config llc90_synthetic --steps 24 --warmup 4 --no-cpu-baseline > $OUT/b_$arm.json 2> $OUT/e_$arm.err || { echo "bench $arm failed"; tail -20 $OUT/e_$arm.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_$arm.json')); k=d['kernel_ms_mean']; print('$arm', 'ms/step %.4f' % d['ms_per_step'], 'phys %.1f phi %.1f us' % (1e3*k['oceanic_phys'], 1e3*k['phi_hyd']))"
done
