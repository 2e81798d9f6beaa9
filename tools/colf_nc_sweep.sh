set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/colfsw
for nc in 16 32 64; do
  MGCM_COLF_NC=$nc timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/colfsw/p$nc -o run --output-format csv -- python3 bench.py --config llc90_synthetic --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/colfsw/b$nc.json 2> gpurun_out/colfsw/e$nc.err || { echo fail $nc; tail -5 gpurun_out/colfsw/e$nc.err; exit 1; }
  python3 - <<PY
import csv, glob
f = glob.glob("gpurun_out/colfsw/p$nc/**/*kernel_stats.csv", recursive=True)[0]
out = {}
for r in csv.DictReader(open(f)):
    n = r["Name"].split("(")[0].replace("mgcm::", "").replace("void ", "")
    if n in ("k_corr_cont", "k_phi_hyd", "k_tracer_impl", "k_sfp_rhs", "k_update_r_star_cg2d_a"): out[n] = round(float(r["AverageNs"]) / 1e3, 1)
print("NC=$nc", out)
PY
done
