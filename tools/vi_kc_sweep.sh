#!/bin/bash
# LLC-90 bench lines of the default VI k-march per MGCM_VI_KC (levels per workgroup).
#   KCS="5 10 17 25"  OUT=gpurun_out/vi_kc
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/vi_kc}
KCS=${KCS:-"5 10 17 25"}
mkdir -p $OUT
for kc in $KCS; do
  MGCM_VI_KC=$kc timeout -k 10 200 python bench.py --config llc90_synthetic --steps 24 --warmup 4 --no-cpu-baseline > $OUT/bench_kc$kc.json 2> $OUT/bench_kc$kc.err || { echo "bench kc $kc failed"; tail -20 $OUT/bench_kc$kc.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_kc$kc.json')); print('kc $kc', 'ms/step %.4f' % d['ms_per_step'], 'mom_step %.1f us' % (1e3*d['kernel_ms_mean']['mom_step']))"
done
