#!/bin/bash
# C2/C3 launch fusions: the whole GPU suite, then the C2 and C3 benches with and without them
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/fuse; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
run() {  # name config steps env...
  local name=$1 c=$2 n=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --config $c --steps $n --warmup 20 --no-cpu-baseline > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python -c "import json; d=json.load(open('$O/$name.json')); k=d['kernel_ms_mean']; print('%-16s step %.4f' % ('$name', d['ms_per_step']), {a: round(b*1e3,1) for a,b in k.items()})"
}
run c2_fused global_ocean.90x40x15 400
run c2_unfused global_ocean.90x40x15 400 MGCM_NO_STEP_FUSE=1
run c3_fused global_ocean.cs32x15 200
run c3_unfused global_ocean.cs32x15 200 MGCM_NO_STEP_FUSE=1
