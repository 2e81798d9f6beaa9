# A/B of where UPDATE_CG2D rides in the fold (MGCM_OPE_AT 1: grids 1+2, 2: grids 2+3), config 2
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ope_at3
MGCM_OPE_AT=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ocean90.py > gpurun_out/ope_at3/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/ope_at3/pytest.log; exit 1; }
tail -1 gpurun_out/ope_at3/pytest.log


for r in 1 2 3; do
  for a in 2 3; do
    MGCM_OPE_AT=$a timeout -k 10 120 python bench.py --steps 400 --warmup 40 --no-cpu-baseline > gpurun_out/ope_at3/b_at${a}_$r.json 2>gpurun_out/ope_at3/err || exit 1
  done
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/ope_at3/b_*.json
