#!/bin/bash
# Round 6: C2's fused grids (k_dt_l1/l2/l3) with their longest bodies dispatched first
# (MGCM_DT_ORDER=1, since folded into MGCM_DT_LAYOUT: the default, =4 the old order -- CALC_PHI_HYD's columns, the tracers' right-hand sides, the implicit
# solves at the head of each grid) against the listed order (0): parity (config 2, 10 steps
# vs the device-order oracle), then C2 bench A/B alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6o}
mkdir -p $OUT
MGCM_DT_ORDER=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ocean90.py -m gpu -x -v -s -k "10_steps" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2 3; do
  for o in 0 1; do
    MGCM_DT_ORDER=$o timeout -k 10 200 python3 bench.py --config global_ocean.90x40x15 --steps 200 --warmup 20 --no-cpu-baseline --no-cs32 > $OUT/c2_o${o}_$rep.json 2> $OUT/c2_o${o}_$rep.err || { echo bench failed; tail -5 $OUT/c2_o${o}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c2_o${o}_$rep.json')); k=d['kernel_ms_mean']; print('C2 order=$o', round(d['ms_per_step'],4), {a: round(b*1e3,1) for a, b in k.items() if b > 0.005})"
  done
done
