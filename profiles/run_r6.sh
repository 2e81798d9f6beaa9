#!/bin/bash
# Round-6 profiles: bench + rocprofv3 kernel stats + FETCH/WRITE PMC passes (with the
# 8-B-lane calibration) per config, each config's kernels alone (--no-cs32), into
# gpurun_out/r6_<tag>/ (copied to profiles/r06/<tag>_final/).
#   bash profiles/run_r6.sh ocean90|cs32x15|llc90 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
for c in "$@"; do
  case $c in
    llc90) CONFIG=llc90_synthetic BENCH_ARGS="--steps 30 --warmup 4 --no-cs32" ;;
    ocean90) CONFIG=global_ocean.90x40x15 BENCH_ARGS="--steps 200 --warmup 20 --no-cs32" ;;
    cs32x15) CONFIG=global_ocean.cs32x15 BENCH_ARGS="--steps 100 --warmup 10 --no-cs32" ;;
    *) echo "unknown config $c"; exit 2 ;;
  esac
  MODE=prof CONFIG=$CONFIG TAG=r6_$c BENCH_ARGS="$BENCH_ARGS" PMC_ARGS="--no-cs32" bash profiles/run_r2.sh || exit 1
done
