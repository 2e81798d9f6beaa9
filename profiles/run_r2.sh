#!/bin/bash
# Round-2 GPU session: parity tests, smoke, bench, rocprofv3 kernel stats, HBM PMC passes
# (with the 8-B-per-lane counter calibration of tools/pmc_calib).
#   MODE=tests|bench|prof|all  CONFIG=<bench --config>  TAG=<profiles/r02 subdir>
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
MODE=${MODE:-all}
CONFIG=${CONFIG:-global_ocean.90x40x15}
TAG=${TAG:-ocean90}
BENCH_ARGS=${BENCH_ARGS:-"--steps 200 --warmup 20"}
PMC_ARGS=${PMC_ARGS:-}   # extra bench arguments of the PMC passes (round 5: --no-cs32)
PT=${PT:-tests}
O=gpurun_out/$TAG
mkdir -p $O
if [ "$MODE" = tests ] || [ "$MODE" = all ]; then
  timeout -k 10 900 python -u -m pytest $PT -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_gpu.log; exit 1; }
  tail -5 $O/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
  cat $O/smoke.log
fi
if [ "$MODE" = bench ] || [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  timeout -k 10 600 python bench.py --config $CONFIG $BENCH_ARGS > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -30 $O/bench.err; exit 1; }
  cat $O/bench.json
fi
if [ "$MODE" = prof ] || [ "$MODE" = all ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config $CONFIG $BENCH_ARGS --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err || { echo rocprof failed; tail -30 $O/prof.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --config $CONFIG --steps 20 --warmup 2 --no-cpu-baseline $PMC_ARGS > $O/pmc_fetch.json 2> $O/pmc_fetch.err || { echo pmc fetch failed; tail -30 $O/pmc_fetch.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --config $CONFIG --steps 20 --warmup 2 --no-cpu-baseline $PMC_ARGS > $O/pmc_write.json 2> $O/pmc_write.err || { echo pmc write failed; tail -30 $O/pmc_write.err; exit 1; }
  if [ -x tools/pmc_calib ]; then
    timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/calib_fetch -o run --output-format csv -- tools/pmc_calib > $O/calib.log 2>&1 || { echo calib fetch failed; tail $O/calib.log; exit 1; }
    timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/calib_write -o run --output-format csv -- tools/pmc_calib >> $O/calib.log 2>&1 || { echo calib write failed; tail $O/calib.log; exit 1; }
    python tools/pmc_summary.py $O/pmc_fetch $O/pmc_write $O/pmc_summary.json $O/calib_fetch $O/calib_write
  else
    python tools/pmc_summary.py $O/pmc_fetch $O/pmc_write $O/pmc_summary.json
  fi
  cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
  echo done
fi
