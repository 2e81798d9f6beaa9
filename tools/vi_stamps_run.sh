set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/vist
MGCM_LIB=mitgcm_amd/_build/diag/libmitgcm_amd_vistamps.so timeout -k 10 200 python bench.py --config llc90_synthetic --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/vist/out.txt 2> gpurun_out/vist/err.txt || { tail -5 gpurun_out/vist/err.txt; exit 1; }
grep -c VISTAMP gpurun_out/vist/out.txt
