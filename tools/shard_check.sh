#!/bin/bash
# The tile-sharded path on one GPU: its GPU tests (gloo ranks sharing cuda:0, RCCL world 1),
# then bench lines of the sharded driver over a one-rank RCCL group beside the resident path
# ($CONFIGS; each step under its own limit, the script stops at the first failure).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-shard_check}
mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parallel.py tests/test_gpu_rccl.py > $O/pytest.log 2>&1
  rc=$?
  tail -3 $O/pytest.log
  grep -E "FAILED|ERROR" $O/pytest.log | head -20
  [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 1; }
fi
for c in ${CONFIGS:-llc90_synthetic global_ocean.cs32x15}; do
  args="--steps 30 --warmup 4"
  [ "$c" = global_ocean.cs32x15 ] && args="--steps 100 --warmup 10"
  for mode in resident shard; do
    extra=""
    [ $mode = shard ] && extra="--shard"
    timeout -k 10 400 python bench.py --config $c $args --no-cpu-baseline $extra > $O/bench_${c}_$mode.json 2> $O/bench_${c}_$mode.err || { echo "bench $c $mode failed"; tail -20 $O/bench_${c}_$mode.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${c}_$mode.json')); print('$c $mode', d['config'].get('cg2d'), 'ms/step %.4f' % d['ms_per_step'], {k: round(v*1e3,1) for k,v in d['kernel_ms_mean'].items()})"
  done
done
