# A/B of where UPDATE_CG2D rides in the fold (MGCM_OPE_AT 1: grids 1+2, 2: grids 2+3), config 2
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ope_at
MGCM_OPE_AT=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ocean90.py > gpurun_out/ope_at/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/ope_at/pytest.log; exit 1; }
tail -1 gpurun_out/ope_at/pytest.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parallel.py tests/test_gpu_rccl.py > gpurun_out/ope_at/pytest_par.log 2>&1 || { echo parallel pytest failed; tail -30 gpurun_out/ope_at/pytest_par.log; exit 1; }
tail -1 gpurun_out/ope_at/pytest_par.log
for r in 1 2 3; do
  for a in 1 2; do
    MGCM_OPE_AT=$a timeout -k 10 120 python bench.py --steps 400 --warmup 40 --no-cpu-baseline > gpurun_out/ope_at/b_at${a}_$r.json 2>gpurun_out/ope_at/err || exit 1
  done
done
grep -o '"ms_per_step": [0-9.]*' gpurun_out/ope_at/b_*.json
