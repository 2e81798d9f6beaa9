#!/bin/bash
# config 2: k_cg2d_bxy geometry variant 0 (2x4 points x 512 threads) vs 1 (2x2 x 1024)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/cgx
for v in 0 1 0 1; do
  MGCM_CGX=$v timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/cgx/b$v.json 2> gpurun_out/cgx/e$v.err || { echo fail; tail -5 gpurun_out/cgx/e$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/cgx/b$v.json')); print('CGX=$v', round(d['ms_per_step'],4), 'cg2d', round(d['kernel_ms_mean']['cg2d']*1e3,1), 'us/it', round(d['roofline']['us_per_iteration'],3))"
done
