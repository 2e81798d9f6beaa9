# The multi-workgroup CG2D's poll loop: the timeout word every 64th pass (default) against every
# pass (lib_old), and no s_sleep between passes (lib_nosleep); parity first
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/mwpoll
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cg2d_mwg.py tests/test_gpu_cs32x15.py tests/test_gpu_cg2d_sr.py > gpurun_out/mwpoll/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/mwpoll/pytest.log; exit 1; }
tail -1 gpurun_out/mwpoll/pytest.log
OUT=gpurun_out/mwpoll CONFIGS="global_ocean.cs32x15 llc90_synthetic" LIBS="default old:mitgcm_amd/_variants/lib_old.so nosleep:mitgcm_amd/_variants/lib_nosleep.so" bash tools/lib_ab.sh
