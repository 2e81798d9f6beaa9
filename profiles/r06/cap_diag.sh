# (round-6 knobs as later consolidated: MGCM_AMD_CAPTURE=multi,debug[,relaxed][,nopool])
#!/bin/bash
# Round 6: where the multi-stream multi-model capture dies (host SIGSEGV, round 5's finding):
# refhost_ref with 4 device models, MGCM_AMD_CAPTURE=multi, one process per runtime setting,
# each stage printed (MGCM_AMD_CAPTURE_DEBUG=1).  Host-process faults only; each run bounded.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6e}
mkdir -p $OUT
timeout -k 10 200 python3 tools/refhost_case.py ref 4 $OUT/case > $OUT/case.log 2>&1 || { echo case setup failed; tail -5 $OUT/case.log; exit 1; }
run() {
  local tag=$1; shift
  env "$@" MGCM_AMD_MODELS=4 MGCM_AMD_EAGER=0 MGCM_CG2D_MWG=0 MGCM_AMD_CAPTURE=multi,debug \
    timeout -k 10 120 mitgcm_amd/fortran/refhost/refhost_ref $OUT/case tests/golden/global_ocean.90x40x15/input > $OUT/$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc: $(grep -c 'capture\[' $OUT/$tag.log) stage lines; last: $(grep 'capture\[' $OUT/$tag.log | tail -1)"
  return 0
}
run default
run pktcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run gq1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1
run relaxed MGCM_AMD_CAPTURE=multi,debug,relaxed
run hwq8 GPU_MAX_HW_QUEUES=8
run nopool MGCM_AMD_CAPTURE=multi,debug,nopool
