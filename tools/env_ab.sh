#!/bin/bash
# generic A/B of an environment switch on one config: ENVVAR=name CONFIG=... STEPS=...
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/envab
c=${CONFIG:-global_ocean.90x40x15}
for v in 0 1 0 1 0 1; do
  if [ $v = 1 ]; then export $ENVVAR=1; else unset $ENVVAR; fi
  timeout -k 10 200 python bench.py --config $c --steps ${STEPS:-300} --warmup 20 --no-cpu-baseline > gpurun_out/envab/b$v.json 2> gpurun_out/envab/e$v.err || { echo fail; tail -5 gpurun_out/envab/e$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/envab/b$v.json')); print('$c $ENVVAR=$v', round(d['ms_per_step'],4), round(d['value'],2))"
done
