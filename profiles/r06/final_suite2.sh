#!/bin/bash
# Round 6: capture diagnosis (stream count), the rest of the -m gpu suite from the refhost
# tests on, smoke, the driver's bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6h}
mkdir -p $OUT
bash profiles/r06/cap_diag2.sh r6f
timeout -k 10 900 python -u -m pytest tests/test_gpu_refhost.py tests/test_gpu_refpin.py tests/test_gpu_restart.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error" $OUT/pytest.log | head; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
grep -a "virtual GPUs:\|step ms one-stream" $OUT/pytest.log | cut -c1-600 | head -30
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo bench failed; tail -5 $OUT/bench_driver.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_driver.json')); print('C2 20 steps', round(d['ms_per_step'],4), round(d['value'],1), 'cs32', round(d['cs32x15']['ms_per_step'],4), 'cpu', d['cpu_baseline']['value'], d['cpu_baseline'].get('all_cores',{}).get('value'), d['cpu_baseline'].get('all_cores',{}).get('tiling'), 'cs32 cpu', d['cs32x15']['cpu_baseline']['value'], d['cs32x15']['cpu_baseline'].get('all_cores',{}).get('value'))"
