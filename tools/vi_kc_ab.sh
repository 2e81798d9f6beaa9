# VI k-march levels per workgroup on LLC-90 (MGCM_VI_KC: default 10, 17, 25)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/vikc
for r in 1 2; do
  for kc in 10 17 25; do
    MGCM_VI_KC=$kc timeout -k 10 200 python bench.py --config llc90_synthetic --steps 30 --warmup 4 --no-cpu-baseline > gpurun_out/vikc/b_kc${kc}_$r.json 2>gpurun_out/vikc/err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/vikc/b_kc${kc}_$r.json')); print($kc, $r, round(d['ms_per_step'],4), round(d['kernel_ms_mean']['mom_step'],4))"
  done
done
