#!/bin/bash
# Round-5 A/B: the VI k-march with its next level staged by LDS-DMA (MGCM_VI_GL=1) against the
# register path, LLC-90 alternating; then the LLC parity tests with the DMA form.
# (the recipe of profiles/r05/vi_gl/; the MGCM_VI_GL variant was measured slower and removed)
#   bash profiles/vi_gl.sh <out-tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
MGCM_VI_GL=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_llc.py \
  -k "vi or None" > $O/llc_parity.log 2>&1; r=$?; tail -2 $O/llc_parity.log
[ $r -eq 0 ] || exit $r
for v in 0 1 0 1 0 1; do
  MGCM_VI_GL=$v timeout -k 10 200 python bench.py --config llc90_synthetic --steps 40 --warmup 4 --no-cs32 \
    --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1])
print('vi_gl=$v', round(d['ms_per_step'],4), 'mom', d['kernel_ms_mean'].get('mom_step'))"
done
