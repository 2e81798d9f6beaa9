#!/bin/bash
# THERMODYNAMICS on the second stream (default) vs serial (MGCM_NO_OVERLAP=1), per config
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/ovl
for c in ${CONFIGS:-global_ocean.90x40x15}; do
for v in 0 1 0 1; do
  if [ $v = 1 ]; then export MGCM_NO_OVERLAP=1; else unset MGCM_NO_OVERLAP; fi
  st=300; [ $c = llc90_synthetic ] && st=30
  timeout -k 10 200 python bench.py --config $c --steps $st --warmup 10 --no-cpu-baseline > gpurun_out/ovl/b$v.json 2> gpurun_out/ovl/e$v.err || { echo fail; tail -5 gpurun_out/ovl/e$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ovl/b$v.json')); print('$c NO_OVERLAP=$v', round(d['ms_per_step'],4), round(d['value'],2))"
done
done
