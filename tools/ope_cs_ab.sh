# UPDATE_CG2D early on the gm_phi path (config 3): parity, then A/B (MGCM_STEP_FUSE 3469 default
# vs 2445 without MG_FUSE_OPE)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ope_cs
MGCM_OPE_GM=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cs32x15.py tests/test_gpu_cube.py tests/test_gpu_options.py tests/test_gpu_cg2d_sr.py > gpurun_out/ope_cs/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/ope_cs/pytest.log; exit 1; }
tail -1 gpurun_out/ope_cs/pytest.log
for r in 1 2 3; do
  for fz in 3469 2445; do
    MGCM_OPE_GM=$([ $fz = 3469 ] && echo 1 || echo 0) MGCM_STEP_FUSE=$fz timeout -k 10 200 python bench.py --config global_ocean.cs32x15 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/ope_cs/b_f${fz}_$r.json 2>gpurun_out/ope_cs/err || exit 1
  done
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/ope_cs/b_*.json
