#!/bin/bash
# k_cg2d_mwg import-polling waves (tools/mwg_npw_build.sh libraries): parity tests with
# one variant, then LLC-90 and cs32x15 bench lines per variant
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/npw}
mkdir -p $OUT
MGCM_LIB=mitgcm_amd/libmitgcm_amd_npw${TESTNPW:-2}.so timeout -k 10 400 python -u -m pytest tests/test_gpu_cg2d_mwg.py tests/test_gpu_cs32x15.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in ${VARS:-def 1 2 4}; do
  lib=mitgcm_amd/libmitgcm_amd.so; [ $v != def ] && lib=mitgcm_amd/libmitgcm_amd_npw$v.so
  for c in llc90_synthetic global_ocean.cs32x15; do
    st=24; [ $c = global_ocean.cs32x15 ] && st=200
    MGCM_LIB=$lib timeout -k 10 200 python bench.py --config $c --steps $st --warmup 10 --no-cpu-baseline > $OUT/b_${v}_$c.json 2> $OUT/e_${v}_$c.err || { echo "bench $v $c failed"; tail -20 $OUT/e_${v}_$c.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b_${v}_$c.json')); print('npw $v $c', 'ms/step %.4f' % d['ms_per_step'], 'cg2d us/it %.3f' % d['roofline']['us_per_iteration'])"
  done
done
