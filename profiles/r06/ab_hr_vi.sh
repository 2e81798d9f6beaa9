#!/bin/bash
# (historical: MGCM_CG2D_HR and MGCM_VI_SPLIT were removed after this A/B -- k_cg2d_hr
# measured slower and was dropped, the VI U-then-V split became the only form)
# Round 6 A/B: CG2D k_cg2d_hr vs k_cg2d_bxy on config 2; VI U/V split variants on LLC-90.
# Parity first (the tests that cover both), then alternating bench runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6b}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ocean90.py tests/test_gpu_latlon.py "tests/test_gpu_llc.py::test_llc30_8_steps_bitexact_vs_device_order_oracle" -x -v -s --timeout 200 --timeout-method thread > $OUT/pytest_ab.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error" $OUT/pytest_ab.log | head; tail -30 $OUT/pytest_ab.log; exit 1; }
tail -1 $OUT/pytest_ab.log
for rep in 1 2; do
  for hr in 1 0; do
    MGCM_CG2D_HR=$hr timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-cs32 > $OUT/c2_hr${hr}_$rep.json 2> $OUT/c2_hr${hr}_$rep.err || { echo bench failed; tail -5 $OUT/c2_hr${hr}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c2_hr${hr}_$rep.json')); r=d['roofline']; print('C2 hr=$hr', round(d['ms_per_step'],4), 'cg2d us/it', round(r['us_per_iteration'],3), r['kernel'])"
  done
done
for rep in 1 2; do
  for sp in 0 1 3; do
    MGCM_VI_SPLIT=$sp timeout -k 10 200 python3 bench.py --config llc90_synthetic --steps 40 --warmup 10 --no-cpu-baseline > $OUT/llc_sp${sp}_$rep.json 2> $OUT/llc_sp${sp}_$rep.err || { echo bench llc failed; tail -5 $OUT/llc_sp${sp}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/llc_sp${sp}_$rep.json')); k=d['kernel_ms_mean']; print('LLC split=$sp', round(d['ms_per_step'],4), 'mom_step ms', round(k['mom_step'],4))"
  done
done
