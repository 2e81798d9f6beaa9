#!/bin/bash
# Round 6: a stand-alone HIP capture across N streams (tools/capture_repro.hip) at N = 2..6, and
# the refhost / refpin / restart GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6k}
mkdir -p $OUT
for nb in "2 4" "3 4" "4 1" "4 4" "4 15" "6 4"; do
  set -- $nb
  timeout -k 10 60 tools/capture_repro $1 $2 > $OUT/repro_$1_$2.log 2>&1
  echo "streams=$1 barriers=$2 rc=$?: $(tail -1 $OUT/repro_$1_$2.log)"
done
timeout -k 10 800 python -u -m pytest tests/test_gpu_refhost.py tests/test_gpu_refpin.py tests/test_gpu_restart.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error" $OUT/pytest.log | head; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
grep -a "virtual GPUs:\|step ms one-stream" $OUT/pytest.log | cut -c1-700 | head -30
