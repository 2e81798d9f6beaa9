#!/bin/bash
# Round 6 (after the knob consolidation): capture diagnosis, then the GPU test files the
# round's changes touch (the rest passed on this tree's kernels in r6g: 131 tests).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6i}
mkdir -p $OUT
bash profiles/r06/cap_diag2.sh r6f
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_latlon.py tests/test_gpu_ocean90.py tests/test_gpu_llc.py tests/test_gpu_refhost.py tests/test_gpu_refpin.py tests/test_gpu_restart.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error" $OUT/pytest.log | head; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
grep -a "gyre 10 steps\|virtual GPUs:\|step ms one-stream" $OUT/pytest.log | cut -c1-700 | head -30
