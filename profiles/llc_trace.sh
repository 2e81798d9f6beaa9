#!/bin/bash
# LLC-90 graph-replay timelines (rocprofv3 kernel trace): overlap forced off / on at VI KC=17
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/llct; mkdir -p $O
MGCM_VI_KC=17 MGCM_NO_OVERLAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/off -o llc -- python bench.py --config llc90_synthetic --steps 10 --warmup 4 --no-cpu-baseline > $O/off.json 2> $O/off.err || { echo "off failed"; tail -5 $O/off.err; exit 1; }
MGCM_VI_KC=17 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/on -o llc -- python bench.py --config llc90_synthetic --steps 10 --warmup 4 --no-cpu-baseline > $O/on.json 2> $O/on.err || { echo "on failed"; tail -5 $O/on.err; exit 1; }
find $O -name "*kernel_trace.csv"
