#!/bin/bash
# Round-5 A/B on LLC-90 of one environment switch (VAR = 0 | 1), alternating, then the LLC
# parity tests with VAR = 1.
#   bash profiles/env_ab2.sh <out-tag> <VAR>
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
V=$2
mkdir -p $O
for v in 0 1 0 1 0 1; do
  env $V=$v timeout -k 10 200 python bench.py --config llc90_synthetic --steps 40 --warmup 4 --no-cs32 \
    --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1])
k=d['kernel_ms_mean']; print('$V=$v', round(d['ms_per_step'],4), {n: round(x, 4) for n, x in k.items() if x})"
done
env $V=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_llc.py \
  > $O/llc_parity.log 2>&1; tail -2 $O/llc_parity.log
