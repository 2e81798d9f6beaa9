#!/bin/bash
# CG2D_SR (useSRCGSolver=1, three barriers per iteration) against the standard CG2D (four),
# config 2: parity tests, then alternating bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/srab
timeout -k 10 300 python -u -m pytest tests/test_gpu_cg2d_sr.py tests/test_gpu_ocean90.py -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/srab/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/srab/pytest.log; exit 1; }
grep -a "CG2D_SR\|passed\|failed" gpurun_out/srab/pytest.log
for v in 1 0 1 0; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --set useSRCGSolver=$v > gpurun_out/srab/b$v.json 2> gpurun_out/srab/e$v.err || { echo fail; tail -5 gpurun_out/srab/e$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/srab/b$v.json')); print('SR=$v', round(d['ms_per_step'],4), round(d['value'],1), 'cg2d', round(d['kernel_ms_mean']['cg2d']*1e3,1), 'its', round(d['cg2d_mean_iters_per_solve'],1), 'us/it', round(d['roofline']['us_per_iteration'],3))"
done
