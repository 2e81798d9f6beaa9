set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/mwst
for c in llc90 cs32x15; do
  MGCM_LIB=mitgcm_amd/_build/diag/libmitgcm_amd_stamps.so timeout -k 10 200 python tools/cg_stamp_run.py $c > gpurun_out/mwst/$c.txt 2>&1 || { tail -5 gpurun_out/mwst/$c.txt; exit 1; }
  grep MWSTAMP gpurun_out/mwst/$c.txt | tail -3
done
