#!/bin/bash
# rocprofv3 kernel stats of a short LLC-90 bench under the given env (ENVS="A=1 B=2")
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/profq}
CONFIG=${CONFIG:-llc90_synthetic}
mkdir -p $OUT
env $ENVS timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --config $CONFIG --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/prof.err || { echo rocprof failed; tail -20 $OUT/prof.err; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    print(r['Name'][:70].ljust(70), r['Calls'], round(float(r['AverageNs'])/1e3,1))"
