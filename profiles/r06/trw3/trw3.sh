#!/bin/bash
# Round 6: C3's k_tr_rhs_pair<true> (186 VGPRs, 2 waves per SIMD: 720 workgroups = 1.41 rounds
# of 512) compiled for 3 waves per SIMD (168 VGPRs, 32 spilled; one round of 768) -- variant
# library mitgcm_amd/_build/diag/libmitgcm_amd_trw3.so via MGCM_LIB: parity (cs32x15 8 steps),
# then C3 bench A/B alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6w}
mkdir -p $OUT
V=$PWD/mitgcm_amd/_build/diag/libmitgcm_amd_trw3.so
MGCM_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_cs32x15.py -m gpu -x -v -s -k "8_steps" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2 3; do
  for v in base trw3; do
    if [ $v = base ]; then unset MGCM_LIB; else export MGCM_LIB=$V; fi
    timeout -k 10 200 python3 bench.py --config global_ocean.cs32x15 --steps 100 --warmup 10 --no-cpu-baseline --no-cs32 > $OUT/c3_${v}_$rep.json 2> $OUT/c3_${v}_$rep.err || { echo bench failed; tail -5 $OUT/c3_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c3_${v}_$rep.json')); print('C3 $v', round(d['ms_per_step'],4), 'temp_step', round(d['kernel_ms_mean'].get('temp_step',0)*1e3,1))"
  done
done
