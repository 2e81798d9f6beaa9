# A/B on LLC-90: the VI k-march's intermediates tail dealt out over the waves (MGCM_VI_M2_VAR 30
# (historical: the var-30 tail and the MGCM_CORR_UNR / MGCM_SFP_UNR variants were measured slower and
# removed after this A/B -- profiles/r04/llc_ab/ holds its results)
# vs 14), the correction pass's level loop unrolled (MGCM_CORR_UNR 1 / 2 / 4) and the halo-ring
# AB2 beside the solve (MGCM_STEP_FUSE 3469 default vs 1421 without MG_FUSE_RING)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/vitail
MGCM_VI_M2_VAR=30 MGCM_CORR_UNR=4 MGCM_SFP_UNR=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_llc.py > gpurun_out/vitail/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/vitail/pytest.log; exit 1; }
tail -1 gpurun_out/vitail/pytest.log
for r in 1 2; do
  for v in "14 1 3469 1" "14 1 1421 1" "30 1 3469 1" "14 4 3469 1" "14 1 3469 4"; do
    set -- $v
    MGCM_VI_M2_VAR=$1 MGCM_CORR_UNR=$2 MGCM_STEP_FUSE=$3 MGCM_SFP_UNR=$4 timeout -k 10 200 python bench.py --config llc90_synthetic --steps 30 --warmup 4 --no-cpu-baseline > gpurun_out/vitail/b_v$1_u$2_f$3_s$4_$r.json 2>gpurun_out/vitail/err || exit 1
  done
done
for f in gpurun_out/vitail/b_*.json; do python -c "import json,sys; d=json.load(open('$f')); k=d['kernel_ms_mean']; print('$f', round(d['ms_per_step'],4), 'mom', round(k['mom_step'],4), 'cont', round(k['continuity'],4), 'sfp', round(k['sfp_rhs'],4))"; done
