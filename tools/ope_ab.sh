set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ope
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ocean90.py tests/test_gpu_refhost.py tests/test_gpu_cg2d_mwg.py > gpurun_out/ope/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/ope/pytest.log; exit 1; }
tail -1 gpurun_out/ope/pytest.log
for r in 1 2; do
  MGCM_STEP_FUSE=397 timeout -k 10 120 python bench.py --steps 400 --warmup 40 --no-cpu-baseline > gpurun_out/ope/b_base_$r.json 2>gpurun_out/ope/err || exit 1
  timeout -k 10 120 python bench.py --steps 400 --warmup 40 --no-cpu-baseline > gpurun_out/ope/b_ope_$r.json 2>gpurun_out/ope/err || exit 1
done
grep -ho '"ms_per_step": [0-9.]*' gpurun_out/ope/b_*.json
