set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/uvab
for v in split nosplit split nosplit; do
  if [ $v = nosplit ]; then export MGCM_MOM_NOSPLIT=1; else unset MGCM_MOM_NOSPLIT; fi
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/uvab/b_$v.json 2> gpurun_out/uvab/e_$v.err || { echo fail; tail -5 gpurun_out/uvab/e_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/uvab/b_$v.json')); print('$v', round(d['ms_per_step'],4), round(d['value'],1), round(d['kernel_ms_mean']['mom_step']*1e3,1))"
done
