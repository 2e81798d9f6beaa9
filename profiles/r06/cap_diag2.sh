#!/bin/bash
# Round 6: the multi-stream capture's fault, placed op by op (MGCM_AMD_CAPTURE_DEBUG=1), at 4
# models (faults) and at 3 (round 5: replays), one run each; host-process faults only.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6f}
mkdir -p $OUT
timeout -k 10 200 python3 tools/refhost_case.py ref 4 $OUT/case > $OUT/case.log 2>&1 || { echo case setup failed; tail -5 $OUT/case.log; exit 1; }
for n in 4 3; do
  MGCM_AMD_MODELS=$n MGCM_AMD_EAGER=0 MGCM_CG2D_MWG=0 MGCM_AMD_CAPTURE=multi MGCM_AMD_CAPTURE_DEBUG=1 \
    timeout -k 10 120 mitgcm_amd/fortran/refhost/refhost_ref $OUT/case tests/golden/global_ocean.90x40x15/input > $OUT/m$n.log 2>&1
  echo "models=$n rc=$?: $(grep -c 'MGCM_AMD ' $OUT/m$n.log) lines"
  grep "MGCM_AMD " $OUT/m$n.log | tail -8
done
