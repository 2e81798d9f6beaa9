#!/bin/bash
# Round-5 GPU check.
#   bash profiles/r5_check.sh <out-tag> bench            -- N=1 bench line (+ cs32x15 sub-record)
#                                                           and the N=2 sharded record over gloo
#   bash profiles/r5_check.sh <out-tag> tests [pytest args]  -- GPU tests (default: all of -m gpu)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
MODE=$2
shift 2
mkdir -p $O
if [ "$MODE" = tests ]; then
  [ $# -gt 0 ] || set -- tests -m gpu
  timeout -k 10 1080 python -u -m pytest -x -v --timeout 600 --timeout-method thread "$@" > $O/pytest.log 2>&1
  rc=$?
  tail -5 $O/pytest.log
  exit $rc
fi
timeout -k 10 300 python bench.py > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
MGCM_SHARD_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 \
  > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { tail -20 $O/bench_n2_gloo.err; exit 1; }
python -c "
import json,sys
for f in ('$O/bench_n1.json','$O/bench_n2_gloo.json'):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d['value'], d['ms_per_step'], 'cs32', (d.get('cs32x15') or {}).get('ms_per_step'))
    for r in d.get('sharded', []): print('  sharded', r)
"
