#!/bin/bash
# VI momentum kernel variants on LLC-90 (eager, event-timed mom_step; env knobs of launch_mom_step)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/vi_sweep; mkdir -p $O
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config llc90_synthetic --steps 10 --warmup 2 --no-cpu-baseline > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python -c "import json; d=json.load(open('$O/$name.json')); k=d['kernel_ms_mean']; print('%-22s step %.4f  mom %.1f us  temp %.1f  cg2d %.1f' % ('$name', d['ms_per_step'], 1e3*k['mom_step'], 1e3*k['temp_step'], 1e3*k['cg2d']))"
}
run base
run var1 MGCM_VI_MARCH_VAR=1
run var2 MGCM_VI_MARCH_VAR=2
run var3 MGCM_VI_MARCH_VAR=3
run kc50 MGCM_VI_KC=50
run kc17 MGCM_VI_KC=17
run kc10 MGCM_VI_KC=10
run level MGCM_VI_KERNEL=level
