#!/bin/bash
# CG2D bxy: the recompute form (RC, default) against the four-barrier form, config 2:
# parity tests then alternating bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/rcab
timeout -k 10 300 python -u -m pytest tests/test_gpu_ocean90.py tests/test_gpu_latlon.py tests/test_gpu_parity.py tests/test_gpu_cg2d_mwg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/rcab/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/rcab/pytest.log; exit 1; }
tail -1 gpurun_out/rcab/pytest.log
for v in 1 0 1 0; do   # 1 = MGCM_CG2D_RC recompute form (opt-in)
  MGCM_CG2D_RC=$v timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/rcab/b$v.json 2> gpurun_out/rcab/e$v.err || { echo fail; tail -5 gpurun_out/rcab/e$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/rcab/b$v.json')); print('RC=$v', round(d['ms_per_step'],4), round(d['value'],1), 'cg2d', round(d['kernel_ms_mean']['cg2d']*1e3,1), 'us/it', round(d['roofline']['us_per_iteration'],3))"
done
