#!/bin/bash
# Round-3 GPU session steps (each under its own time limit; see profiles/run_r2.sh for MODE).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
exec_step() { MODE=$1 CONFIG=$2 TAG=$3 BENCH_ARGS="$4" bash profiles/run_r2.sh; }
case "${1:-head}" in
  llc90) exec_step prof llc90_synthetic r3_llc90 "--steps 30 --warmup 4" ;;
  tests) exec_step tests global_ocean.90x40x15 r3_tests "" ;;
  *) echo "unknown step $1"; exit 2 ;;
esac
