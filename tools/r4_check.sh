#!/bin/bash
# Round-4 checkpoint: the whole GPU suite, then config 2 and LLC-90 bench lines (each step under
# its own limit; the script stops at the first failure).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4_check}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit 1; }
for c in ${CONFIGS:-global_ocean.90x40x15}; do
  args="--steps 30 --warmup 4"
  [ "$c" = global_ocean.90x40x15 ] && args="--steps 200 --warmup 20"
  [ "$c" = global_ocean.cs32x15 ] && args="--steps 100 --warmup 10"
  timeout -k 10 600 python bench.py --config $c $args --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail -20 $O/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$c.json')); print('$c', 'ms/step %.4f' % d['ms_per_step'], 'value %.1f' % d['value'], {k: round(v*1e3,1) for k,v in d['kernel_ms_mean'].items()})"
done
