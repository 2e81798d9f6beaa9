set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/ab2
timeout -k 10 500 python -u -m pytest tests/test_gpu_llc.py tests/test_gpu_ocean90.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab2/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/ab2/pytest.log; exit 1; }
tail -1 gpurun_out/ab2/pytest.log
for rep in 1 2; do
 for arm in "MGCM_STEP_FUSE=13" "MGCM_STEP_FUSE=77"; do
  env $arm timeout -k 10 200 python bench.py --config llc90_synthetic --steps 24 --warmup 4 --no-cpu-baseline > gpurun_out/ab2/b.json 2> gpurun_out/ab2/e.err || { tail -20 gpurun_out/ab2/e.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab2/b.json')); print('llc $arm', 'ms/step %.4f' % d['ms_per_step'])"
 done
 for arm in "MGCM_CORR_NC=16" "MGCM_CORR_NC=32"; do
  env $arm timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/ab2/b.json 2> gpurun_out/ab2/e.err || { tail -20 gpurun_out/ab2/e.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab2/b.json')); print('c2 $arm', 'ms/step %.4f' % d['ms_per_step'])"
 done
done
