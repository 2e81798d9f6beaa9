#!/bin/bash
# Round 6: the whole -m gpu suite, smoke, and the driver's bench line (20 steps).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6z}
mkdir -p $OUT
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error" $OUT/pytest.log | head; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo bench failed; tail -5 $OUT/bench_driver.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_driver.json')); print('C2 20 steps', round(d['ms_per_step'],4), round(d['value'],1), 'cs32', round(d['cs32x15']['ms_per_step'],4))"
