#!/bin/bash
# Round 6 final profiles, second pass (after the one-kernel tracer solve became LLC-90's
# default): bench + rocprofv3 kernel stats + PMC passes for llc90 and cs32x15.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
bash profiles/run_r6.sh llc90 cs32x15 > gpurun_out/r6_prof2.log 2>&1 || { echo profiles failed; tail -20 gpurun_out/r6_prof2.log; exit 1; }
for c in llc90 cs32x15; do python3 -c "import json; d=json.load(open('gpurun_out/r6_$c/bench.json')); print('$c', round(d['ms_per_step'],4), round(d['value'],2))"; done
