set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/full
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/full/pytest.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error" gpurun_out/full/pytest.log | head; tail -30 gpurun_out/full/pytest.log; exit 1; }
tail -1 gpurun_out/full/pytest.log
for c in global_ocean.cs32x15 llc90_synthetic; do
  st=200; [ $c = llc90_synthetic ] && st=30
  timeout -k 10 300 python bench.py --config $c --steps $st --warmup 10 --no-cpu-baseline > gpurun_out/full/b_$c.json 2> gpurun_out/full/e_$c.err || { echo bench $c failed; tail -5 gpurun_out/full/e_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/full/b_$c.json')); print('$c', round(d['ms_per_step'],4), round(d['value'],2), 'cg2d', round(d['kernel_ms_mean']['cg2d']*1e3,1), 'us/it', round(d['roofline']['us_per_iteration'],3))"
done
