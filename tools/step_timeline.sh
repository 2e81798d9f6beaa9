#!/bin/bash
# kernel-trace of a short bench run + one step's timeline (tools/step_timeline.py) under ENVS
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/tl}
CONFIG=${CONFIG:-global_ocean.90x40x15}
mkdir -p $OUT
env $ENVS timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 bench.py --config $CONFIG --steps ${STEPS:-20} --warmup 4 --no-cpu-baseline > $OUT/bench.json 2> $OUT/prof.err || { echo rocprof failed; tail -20 $OUT/prof.err; exit 1; }
python3 tools/step_timeline.py $OUT/prof ${FIRST:-k_oceanic_phys} > $OUT/timeline.txt && cat $OUT/timeline.txt
