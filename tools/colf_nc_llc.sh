#!/bin/bash
# LLC-90 bench lines per MGCM_COLF_NC (column-frame width of every column kernel), with the
# LLC parity tests first
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/colfnc}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_llc.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_llc.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_llc.log; exit 1; }
tail -1 $OUT/pytest_llc.log
for nc in ${NCS:-16 32}; do
  MGCM_COLF_NC=$nc timeout -k 10 200 python bench.py --config llc90_synthetic --steps 24 --warmup 4 --no-cpu-baseline > $OUT/b_$nc.json 2> $OUT/e_$nc.err || { echo "bench $nc failed"; tail -20 $OUT/e_$nc.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_$nc.json')); k=d['kernel_ms_mean']; print('nc $nc', 'ms/step %.4f' % d['ms_per_step'], {a: round(1e3*b, 1) for a, b in k.items()})"
done
