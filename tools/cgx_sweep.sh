set -e
mkdir -p gpurun_out/cgx
for v in 0 1 2 3 4 5; do
  MGCM_CGX=$v timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/cgx/v$v.json 2> gpurun_out/cgx/v$v.err || echo "v$v failed"
done
