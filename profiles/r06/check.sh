#!/bin/bash
# Round 6 GPU check: the -m gpu suite (digits printed with -s), the default bench line, and the
# self-spawned N = 2 rehearsal (gloo, both ranks on the one GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6a}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
grep -a "worst\|digits" $OUT/pytest.log | head -40
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo bench failed; tail -5 $OUT/bench_n1.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_n1.json')); print('C2', round(d['ms_per_step'],4), round(d['value'],1), 'cs32', round(d['cs32x15']['ms_per_step'],4), 'cpu', d['cpu_baseline']['value'], d['cpu_baseline'].get('all_cores',{}).get('value'))"
MGCM_SHARD_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_n2.json 2> $OUT/bench_n2.err || { echo bench n2 failed; tail -5 $OUT/bench_n2.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_n2.json')); print('N2', d['n_gpus'], d['distinct_gpus'], round(d['value'],1), [(r['config'], r.get('ms_per_step'), r.get('error')) for r in d.get('sharded', [])])"
