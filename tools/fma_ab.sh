set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
for fm in 0 1 0 1; do
  MGCM_CG2D_FMA=$fm timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/fma$fm.json 2>gpurun_out/fma.err || { tail gpurun_out/fma.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/fma$fm.json')); print('FMA=$fm', round(d['ms_per_step'],4), round(d['value'],1), d['roofline']['us_per_iteration'], d['cg2d_mean_iters_per_solve'])"
done
