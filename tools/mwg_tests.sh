# The multi-workgroup CG2D's GPU tests (cs32x15 / LLC / sharded device solve) after a build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/mwg_tests
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cg2d_mwg.py tests/test_gpu_cs32x15.py tests/test_gpu_cg2d_sr.py tests/test_gpu_llc.py tests/test_gpu_parallel.py -k "not gyre" > gpurun_out/mwg_tests/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/mwg_tests/pytest.log; exit 1; }
tail -1 gpurun_out/mwg_tests/pytest.log
timeout -k 10 200 python bench.py --config global_ocean.cs32x15 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/mwg_tests/b_cs32.json 2>gpurun_out/mwg_tests/err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/mwg_tests/b_cs32.json')); print('cs32', round(d['ms_per_step'],4), round(d['roofline']['us_per_iteration'],3))"
