#!/bin/bash
# SQ counters and HBM bytes of the VI momentum kernel variants on LLC-90 (one --pmc pass each).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/vipmc}
mkdir -p $OUT
for kern in ${KERNELS:-level march:25}; do
  kc=${kern#*:}; [ "$kc" = "$kern" ] && kc=0; kn=${kern%%:*}
  export MGCM_VI_KC=$kc MGCM_VI_KERNEL=$kn
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $OUT/sq_${kn}_$kc -o run --output-format csv -- python3 bench.py --config llc90_synthetic --steps 4 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/sq_${kn}_$kc.err || { echo "sq $kern failed"; tail -5 $OUT/sq_${kn}_$kc.err; exit 1; }
  python tools/sq_summary.py $OUT/sq_${kn}_$kc | grep -E "kernel|k_mom_vi"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fe_${kn}_$kc -o run --output-format csv -- python3 bench.py --config llc90_synthetic --steps 4 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/fe_${kn}_$kc.err || { echo "fetch $kern failed"; exit 1; }
  python - <<PY
import csv, glob, collections
f = glob.glob("$OUT/fe_${kn}_$kc/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("mgcm::", "").replace("void ", "")
    if "k_mom_vi" in k: acc[k].append(float(r["Counter_Value"]))
for k, v in acc.items(): print("  FETCH_SIZE %s: %.1f MB/launch (raw KB, n=%d)" % (k, sum(v) / len(v) / 1024.0, len(v)))
PY
done
