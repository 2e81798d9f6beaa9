#!/bin/bash
# LLC-90 graph-replay timelines (rocprofv3 kernel trace) of the candidate step layouts
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/llct; mkdir -p $O
tr() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$name -o llc -- python bench.py --config llc90_synthetic --steps 10 --warmup 4 --no-cpu-baseline > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
}
tr at1s MGCM_THERMO_AT=1 MGCM_TRACER_PAIR=0 MGCM_TR_KC=5 MGCM_VI_KC=10
tr at1p MGCM_THERMO_AT=1 MGCM_TR_KC=5 MGCM_VI_KC=10
