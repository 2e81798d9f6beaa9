#!/bin/bash
# config 2 bench lines, repeated (variance check for small step-time changes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/c2rep
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/c2rep/b$r.json 2> gpurun_out/c2rep/e$r.err || { echo fail; tail -5 gpurun_out/c2rep/e$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c2rep/b$r.json')); print('run $r', round(d['ms_per_step'],4), round(d['value'],1))"
done
