#!/bin/bash
# Whole GPU suite + smoke, then every BASELINE config's bench at the defaults
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/full; mkdir -p $O
timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for c in global_ocean.90x40x15 global_ocean.cs32x15 llc90_synthetic baroclinic_gyre_dst3; do
  args="--steps 30 --warmup 4"
  [ "$c" = global_ocean.90x40x15 ] && args="--steps 400 --warmup 20"
  [ "$c" = global_ocean.cs32x15 ] && args="--steps 200 --warmup 10"
  [ "$c" = baroclinic_gyre_dst3 ] && args="--steps 400 --warmup 20"
  timeout -k 10 600 python bench.py --config $c $args --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail -20 $O/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$c.json')); print('$c', 'ms/step %.4f' % d['ms_per_step'], d['thermo_overlap'])"
done
