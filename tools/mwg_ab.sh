#!/bin/bash
# k_cg2d_mwg change check: the multi-workgroup CG2D parity tests (single process, LLC,
# cs32x15, device CG2D across processes), then LLC-90 and cs32x15 bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/mwgab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_cg2d_mwg.py tests/test_gpu_cs32x15.py tests/test_gpu_llc.py "tests/test_gpu_parallel.py::test_device_cg2d_across_processes" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for c in llc90_synthetic global_ocean.cs32x15; do
    st=24; [ $c = global_ocean.cs32x15 ] && st=200
    timeout -k 10 200 python bench.py --config $c --steps $st --warmup 10 --no-cpu-baseline > $OUT/b_$c.json 2> $OUT/e_$c.err || { echo "bench $c failed"; tail -20 $OUT/e_$c.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b_$c.json')); print('$c', 'ms/step %.4f' % d['ms_per_step'], 'cg2d us/it %.3f' % d['roofline']['us_per_iteration'])"
  done
done
