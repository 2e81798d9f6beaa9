#!/bin/bash
# Round-3 GPU session steps (each under its own time limit; see profiles/run_r2.sh for MODE).
#   bash profiles/run_r3.sh tests|llc90|ocean90|cs32x15|head
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
exec_step() { MODE=$1 CONFIG=$2 TAG=$3 BENCH_ARGS="$4" bash profiles/run_r2.sh; }
case "${1:-head}" in
  llc90) exec_step prof llc90_synthetic r3_llc90 "--steps 30 --warmup 4" ;;
  ocean90) exec_step prof global_ocean.90x40x15 r3_ocean90 "--steps 200 --warmup 20" ;;
  cs32x15) exec_step prof global_ocean.cs32x15 r3_cs32x15 "--steps 100 --warmup 10" ;;
  tests) exec_step tests global_ocean.90x40x15 r3_tests "" ;;
  head) exec_step tests global_ocean.90x40x15 r3_tests "" &&
        exec_step prof llc90_synthetic r3_llc90 "--steps 30 --warmup 4" ;;
  *) echo "unknown step $1"; exit 2 ;;
esac
