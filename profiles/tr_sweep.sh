#!/bin/bash
# Tracer column kernel A/B on LLC-90 (+ the VI variants that changed the step), after the parity tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/tr_sweep; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_llc.py tests/test_gpu_3d.py tests/test_gpu_latlon.py > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config llc90_synthetic --steps 20 --warmup 4 --no-cpu-baseline > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python -c "import json; d=json.load(open('$O/$name.json')); k=d['kernel_ms_mean']; print('%-22s step %.4f  mom %.1f us  temp %.1f  cg2d %.1f ovl %s' % ('$name', d['ms_per_step'], 1e3*k['mom_step'], 1e3*k['temp_step'], 1e3*k['cg2d'], d['thermo_overlap']))"
}
run col
run col4 MGCM_TRACER_COL=4
run nocol MGCM_TRACER_NOCOL=1
run col_var3 MGCM_VI_MARCH_VAR=3
run col_var3_kc17 MGCM_VI_MARCH_VAR=3 MGCM_VI_KC=17
run col_kc17 MGCM_VI_KC=17
