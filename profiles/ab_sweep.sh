#!/bin/bash
# A/B sweep: C2 launch-fusion masks (MGCM_STEP_FUSE) and LLC-90 VI k-chunk sizes
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
run() {  # name config steps env...
  local name=$1 c=$2 n=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --config $c --steps $n --warmup 20 --no-cpu-baseline > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python -c "import json; d=json.load(open('$O/$name.json')); k=d['kernel_ms_mean']; print('%-16s step %.4f' % ('$name', d['ms_per_step']), {a: round(b*1e3,1) for a,b in k.items()})"
}
for mk in 0 1 2 4 8 13 15; do run c2_m$mk global_ocean.90x40x15 400 MGCM_STEP_FUSE=$mk; done
run c2_m13b global_ocean.90x40x15 400 MGCM_STEP_FUSE=13
run c2_m0b global_ocean.90x40x15 400 MGCM_STEP_FUSE=0
for kc in 10 13 17 25; do run llc_kc$kc llc90_synthetic 20 MGCM_VI_KC=$kc; done
run llc_var3_kc13 llc90_synthetic 20 MGCM_VI_KC=13 MGCM_VI_MARCH_VAR=3
# the graph-replayed LLC-90 step's timeline (per-dispatch start/end) for the gap analysis
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o llc -- python bench.py --config llc90_synthetic --steps 10 --warmup 4 --no-cpu-baseline > $O/trace_bench.json 2> $O/trace_bench.err || { echo "trace failed"; tail -5 $O/trace_bench.err; exit 1; }
find $O/trace -name "*.csv" | head
