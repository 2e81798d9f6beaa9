#!/bin/bash
# cs32x15 (6 parts): k_cg2d_mwg parts pinned to one XCD (default for <= 32 parts) vs spread
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/spread
for v in 1 0 1 0; do
  if [ $v = 1 ]; then export MGCM_CG2D_SPREAD=1; else unset MGCM_CG2D_SPREAD; fi
  timeout -k 10 200 python bench.py --config global_ocean.cs32x15 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/spread/b$v.json 2> gpurun_out/spread/e$v.err || { echo fail; tail -5 gpurun_out/spread/e$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/spread/b$v.json')); print('SPREAD=$v', round(d['ms_per_step'],4), 'cg2d', round(d['kernel_ms_mean']['cg2d']*1e3,1), 'us/it', round(d['roofline']['us_per_iteration'],3))"
done
