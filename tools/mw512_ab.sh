# The multi-workgroup CG2D at 512 threads x 1 point per part (twice the parts) against the
# default 1024 x 1; parity of the variant first
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/mw512
MGCM_LIB=$PWD/mitgcm_amd/_variants/lib_512x1.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cg2d_mwg.py tests/test_gpu_cs32x15.py > gpurun_out/mw512/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/mw512/pytest.log; exit 1; }
tail -1 gpurun_out/mw512/pytest.log
OUT=gpurun_out/mw512 CONFIGS="global_ocean.cs32x15 llc90_synthetic" LIBS="default w512:mitgcm_amd/_variants/lib_512x1.so" bash tools/lib_ab.sh
for f in gpurun_out/mw512/b_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f'.split('/')[-1], round(d['ms_per_step'],4), round(d['roofline']['us_per_iteration'],3), d['roofline']['cus_used'])"; done
