#!/bin/bash
# Round-2 end-of-session GPU pass at HEAD: the whole -m gpu suite and smoke once, then for
# each BASELINE device config a bench line, rocprofv3 kernel stats and the FETCH/WRITE PMC
# passes (profiles/run_r2.sh MODE=prof), each step under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
MODE=tests CONFIG=global_ocean.90x40x15 TAG=head bash profiles/run_r2.sh || exit 1
MODE=prof CONFIG=global_ocean.90x40x15 TAG=ocean90 bash profiles/run_r2.sh || exit 1
MODE=prof CONFIG=global_ocean.cs32x15 TAG=cs32x15 BENCH_ARGS="--steps 100 --warmup 10" bash profiles/run_r2.sh || exit 1
MODE=prof CONFIG=llc90_synthetic TAG=llc90 BENCH_ARGS="--steps 30 --warmup 4" bash profiles/run_r2.sh || exit 1
