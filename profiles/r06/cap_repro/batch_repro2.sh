#!/bin/bash
# Round 6: variants of the stand-alone N-stream capture (tools/capture_repro.hip), run in order
# until the first one that does not exit 0 (nothing more runs on the GPU after a crash).
# Each argument is "HWQ N B what mode" (HWQ = GPU_MAX_HW_QUEUES for that run).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/$1
shift
mkdir -p $OUT
for v in "$@"; do
  set -- $v
  log=$OUT/repro_q$1_$2_$3_$4_$5.log
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 60 tools/capture_repro $2 $3 $4 $5 > $log 2>&1
  rc=$?
  echo "hwq=$1 streams=$2 barriers=$3 ops=$4 mode=$5 rc=$rc: $(tail -1 $log)"
  [ $rc -eq 0 ] || exit 0
done
