#!/bin/bash
# A/B of the VI momentum kernels on the GPU box: parity tests with the k-march forced, then
# LLC-90 bench lines per kernel.  KERNELS entries: level | march:KC:VAR (VAR = k_mom_vi_march
# template variant, MGCM_VI_MARCH_VAR: 0 PF=0 CREG=0, 1 PF CREG, 2 PF, 3 CREG).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/viab}
mkdir -p $OUT
if [ "${TESTS:-1}" = 1 ]; then
  MGCM_VI_KERNEL=march timeout -k 10 300 python -u -m pytest tests/test_gpu_llc.py tests/test_gpu_cs32x15.py tests/test_gpu_options.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_march.log 2>&1 || { echo "pytest (march) failed"; tail -40 $OUT/pytest_march.log; exit 1; }
  tail -2 $OUT/pytest_march.log
fi
for kern in ${KERNELS:-level march:13:0}; do
  IFS=: read kn kc var <<< "$kern"
  MGCM_VI_KC=${kc:-0} MGCM_VI_KERNEL=$kn MGCM_VI_MARCH_VAR=${var:-0} timeout -k 10 200 python bench.py --config llc90_synthetic --steps 24 --warmup 4 --no-cpu-baseline > $OUT/bench_$kern.json 2> $OUT/bench_$kern.err || { echo "bench $kern failed"; tail -20 $OUT/bench_$kern.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$kern.json')); print('$kern', round(d['ms_per_step'],4), 'ms/step', {k: round(v*1e3,1) for k,v in d['kernel_ms_mean'].items() if k in ('mom_step','cg2d','temp_step')})"
done
