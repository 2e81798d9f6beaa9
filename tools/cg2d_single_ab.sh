#!/bin/bash
# cs32x15 (6 x 32^2 = 6144 CG2D points): the generic single-workgroup CG2D (MGCM_CG2D_SINGLE=1)
# against the multi-workgroup default.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/singab
for v in 1 0; do
  MGCM_CG2D_SINGLE=$v timeout -k 10 200 python bench.py --config global_ocean.cs32x15 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/singab/b$v.json 2> gpurun_out/singab/e$v.err || { echo fail; tail -5 gpurun_out/singab/e$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/singab/b$v.json')); print('SINGLE=$v', round(d['ms_per_step'],4), round(d['value'],1), 'cg2d', round(d['kernel_ms_mean']['cg2d']*1e3,1), 'its', round(d['cg2d_mean_iters_per_solve'],1), 'us/it', round(d['roofline']['us_per_iteration'],3))"
done
