set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
for nc in 16 32 64; do
  MGCM_COLF_NC=$nc timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sweep/nc$nc -o run --output-format csv -- python3 bench.py --config llc90_synthetic --steps 24 --warmup 2 --no-cpu-baseline > gpurun_out/sweep/nc$nc.json 2> gpurun_out/sweep/nc$nc.err || { echo fail $nc; tail gpurun_out/sweep/nc$nc.err; exit 1; }
  python - <<PY
import csv, glob
f = glob.glob("gpurun_out/sweep/nc$nc/**/*kernel_stats.csv", recursive=True)[0]
print("NC=$nc", " ".join("%s=%.1f" % (r["Name"].split("(")[0].replace("mgcm::", "").replace("void ", ""), float(r["AverageNs"]) / 1e3) for r in csv.DictReader(open(f)) if any(x in r["Name"] for x in ("impl", "corr", "phi_hyd", "sfp", "tracer_rhs"))))
PY
done
