#!/bin/bash
# (historical: MGCM_AMD_CAPTURE_POOL=0 is now MGCM_AMD_CAPTURE=multi,nopool)
# Round 6: (1) k_cg2d_bxy per-phase s_memtime stamps on config 2 (diagnostic library);
# (2) the multi-model step captured across the models' own streams with per-record events
# (MGCM_AMD_CAPTURE=multi), 4 and 6 models, bit-identical to the one-stream graph;
# (3) the same 4-model capture with the event pool OFF (events re-recorded, round 5's form),
# last, its exit status recorded (a host-process SIGSEGV there is the round-5 finding).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6c}
mkdir -p $OUT
MGCM_LIB=mitgcm_amd/_build/diag/libmitgcm_amd_stamps.so timeout -k 10 120 python3 tools/cg_stamp_run.py ocean90 > $OUT/stamps_ocean90.log 2>&1 || { echo stamps failed; tail -5 $OUT/stamps_ocean90.log; exit 1; }
grep CGSTAMP $OUT/stamps_ocean90.log | head -4
timeout -k 10 600 python -u -m pytest tests/test_gpu_refhost.py -k "multistream or virtual_gpus" -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_cap.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error\|returncode" $OUT/pytest_cap.log | head; tail -30 $OUT/pytest_cap.log; exit 1; }
tail -1 $OUT/pytest_cap.log
grep -a "step ms one-stream\|virtual GPUs:" $OUT/pytest_cap.log
MGCM_AMD_CAPTURE_POOL=0 timeout -k 10 300 python -u -m pytest "tests/test_gpu_refhost.py::test_refhost_multistream_capture[ref-4]" -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_cap_nopool.log 2>&1
echo "pool off rc=$?"
grep -a "returncode\|-11\|passed\|failed" $OUT/pytest_cap_nopool.log | tail -5
