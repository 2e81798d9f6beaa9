#!/bin/bash
# CALC_PHI_HYD column frame width on LLC-90 (MGCM_PHI_NC columns per workgroup), bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/phinc}
mkdir -p $OUT
for nc in ${NCS:-16 32 64}; do
  MGCM_PHI_NC=$nc timeout -k 10 200 python bench.py --config llc90_synthetic --steps 24 --warmup 4 --no-cpu-baseline > $OUT/b_$nc.json 2> $OUT/e_$nc.err || { echo "bench $nc failed"; tail -20 $OUT/e_$nc.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_$nc.json')); k=d['kernel_ms_mean']; print('nc $nc', 'ms/step %.4f' % d['ms_per_step'], 'phi %.1f us' % (1e3*k['phi_hyd']))"
done
