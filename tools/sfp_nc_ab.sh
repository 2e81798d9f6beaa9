# CALC_DIV_GHAT column frame width on LLC-90 (MGCM_SFP_NC 16 default, 32, 64)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sfpnc
MGCM_SFP_NC=32 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_llc.py -k "None" > gpurun_out/sfpnc/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/sfpnc/pytest.log; exit 1; }
tail -1 gpurun_out/sfpnc/pytest.log
for r in 1 2; do
  for nc in 16 32 64; do
    MGCM_SFP_NC=$nc timeout -k 10 200 python bench.py --config llc90_synthetic --steps 30 --warmup 4 --no-cpu-baseline > gpurun_out/sfpnc/b_nc${nc}_$r.json 2>gpurun_out/sfpnc/err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/sfpnc/b_nc${nc}_$r.json')); print($nc, $r, round(d['ms_per_step'],4), round(d['kernel_ms_mean']['sfp_rhs'],4))"
  done
done
for r in 1 2; do
  for nc in 32 64 16; do
    MGCM_CORR_NC=$nc timeout -k 10 200 python bench.py --config llc90_synthetic --steps 30 --warmup 4 --no-cpu-baseline > gpurun_out/sfpnc/b_corr${nc}_$r.json 2>gpurun_out/sfpnc/err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/sfpnc/b_corr${nc}_$r.json')); print('corr', $nc, $r, round(d['ms_per_step'],4), round(d['kernel_ms_mean']['continuity'],4))"
  done
done
