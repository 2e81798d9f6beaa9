# (round-6 knobs as later consolidated: MGCM_AMD_CAPTURE=multi,debug[,relaxed][,nopool])
#!/bin/bash
# Round 6: the multi-stream capture's fault, placed op by op (MGCM_AMD_CAPTURE_DEBUG=1), at 4
# models (faults) and at 3 (round 5: replays), one run each; host-process faults only.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6f}
mkdir -p $OUT
CASE=/tmp/refhost_case_r6   # (kept out of gpurun_out: ~40 MB)
timeout -k 10 200 python3 tools/refhost_case.py ref 4 $CASE > $OUT/case.log 2>&1 || { echo case setup failed; tail -5 $OUT/case.log; exit 1; }
# 4 models (faults), 3 (replays), and 4 models with the THERMODYNAMICS overlap off (each model
# then brings one stream into the capture instead of two)
for cfg in "4 1" "3 1" "4 0"; do
  set -- $cfg
  MGCM_OVERLAP=$2 MGCM_AMD_MODELS=$1 MGCM_AMD_EAGER=0 MGCM_CG2D_MWG=0 MGCM_AMD_CAPTURE=multi,debug \
    timeout -k 10 120 mitgcm_amd/fortran/refhost/refhost_ref $CASE tests/golden/global_ocean.90x40x15/input > $OUT/m$1_ovl$2.log 2>&1
  echo "models=$1 overlap=$2 rc=$?: $(grep -c 'MGCM_AMD ' $OUT/m$1_ovl$2.log) lines"
  grep "MGCM_AMD capture\|MGCM_AMD   op" $OUT/m$1_ovl$2.log | tail -4
done
