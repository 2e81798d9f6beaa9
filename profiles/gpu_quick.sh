#!/bin/bash
# Quick GPU check: selected parity tests then short benches (each step under its own limit).
#   TESTS="tests/a.py tests/b.py" CONFIGS="llc90_synthetic global_ocean.90x40x15" TAG=name
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${TAG:-quick}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
for c in $CONFIGS; do
  args="--steps 30 --warmup 4"
  [ "$c" = global_ocean.90x40x15 ] && args="--steps 200 --warmup 20"
  [ "$c" = global_ocean.cs32x15 ] && args="--steps 100 --warmup 10"
  timeout -k 10 600 python bench.py --config $c $args --no-cpu-baseline $BENCH_EXTRA > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail -20 $O/bench_$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_$c.json')); print('$c', 'ms/step %.4f' % d['ms_per_step'], {k: round(v*1e3,1) for k,v in d['kernel_ms_mean'].items()}, 'overlap', d['thermo_overlap'])"
done
