#!/bin/bash
# k_cg2d_mwg workgroup geometry A/B (tools/mwg_build_variant.sh builds the variants):
# parity of each variant, then cs32x15 and LLC-90 bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/mwab
for v in ${VARIANTS:-256x4 512x2 512x4 1024x2}; do
  lib=mitgcm_amd/libmitgcm_amd_mw$v.so; [ $v = 256x4 ] && lib=mitgcm_amd/libmitgcm_amd.so
  MGCM_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_cg2d_mwg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/mwab/pytest_$v.log 2>&1 || { echo pytest $v failed; tail -20 gpurun_out/mwab/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/mwab/pytest_$v.log)"
  for c in global_ocean.cs32x15 llc90_synthetic; do
    st=100; [ $c = llc90_synthetic ] && st=30
    MGCM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config $c --steps $st --warmup 4 --no-cpu-baseline > gpurun_out/mwab/b_${v}_$c.json 2> gpurun_out/mwab/e_${v}_$c.err || { echo bench $v $c failed; tail -5 gpurun_out/mwab/e_${v}_$c.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/mwab/b_${v}_$c.json')); print('$v $c', round(d['ms_per_step'],4), 'cg2d', round(d['kernel_ms_mean']['cg2d']*1e3,1), 'its', round(d['cg2d_mean_iters_per_solve'],1), 'us/it', round(d['roofline']['us_per_iteration'],3))"
  done
done
