#!/bin/bash
# k_mom_vi_m2 (compile-time specialised VI k-march) vs the generic k_mom_vi_march on LLC-90:
# the LLC parity tests, then one bench line per arm (eager kernel means in kernel_ms_mean).
#   ARMS="m2:0 m2:3 gen:0"  (kind:variant, m2 MGCM_VI_M2_VAR bit mask, gen MGCM_VI_MARCH_VAR)   OUT=gpurun_out/vi_m2
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/vi_m2}
ARMS=${ARMS:-"m2:0 m2:3 gen:0"}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_llc.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_llc.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_llc.log; exit 1; }
tail -2 $OUT/pytest_llc.log
for arm in $ARMS; do
  kind=${arm%%:*}; var=${arm##*:}
  m2=1; [ "$kind" = gen ] && m2=0
  MGCM_VI_M2=$m2 MGCM_VI_M2_VAR=$var MGCM_VI_MARCH_VAR=$var timeout -k 10 200 python bench.py --config llc90_synthetic --steps 24 --warmup 4 --no-cpu-baseline > $OUT/bench_$kind$var.json 2> $OUT/bench_$kind$var.err || { echo "bench $arm failed"; tail -20 $OUT/bench_$kind$var.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$kind$var.json')); print('$arm', 'ms/step %.4f' % d['ms_per_step'], 'mom_step %.1f us' % (1e3*d['kernel_ms_mean']['mom_step']))"
done
