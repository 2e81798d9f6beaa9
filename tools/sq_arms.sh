#!/bin/bash
# SQ counter passes per VI-kernel arm on LLC-90 (tools/sq_summary.py per pass).
#   ARMS="m2:3 gen:0"   OUT=gpurun_out/sq_arms
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/sq_arms}
ARMS=${ARMS:-"m2:3 gen:0"}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" $OUT/avail.txt | sort -u > $OUT/sq_avail.txt || true
P1="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
for arm in $ARMS; do
  kind=${arm%%:*}; var=${arm##*:}
  m2=1; [ "$kind" = gen ] && m2=0
  for pn in 1 2; do
    eval "PC=\$P$pn"
    ok=1; for c in $PC; do grep -qx "$c" $OUT/sq_avail.txt || { echo "counter $c not listed"; ok=0; }; done
    [ $ok = 1 ] || continue
    MGCM_VI_M2=$m2 MGCM_VI_M2_VAR=$var MGCM_VI_MARCH_VAR=$var timeout -s KILL 180 rocprofv3 --pmc $PC -d $OUT/p${pn}_$kind$var -o run --output-format csv -- python3 bench.py --config llc90_synthetic --steps 6 --warmup 1 --no-cpu-baseline > $OUT/b${pn}_$kind$var.json 2> $OUT/p${pn}_$kind$var.err || { echo "pmc $arm pass $pn failed"; tail -5 $OUT/p${pn}_$kind$var.err; exit 1; }
    python tools/sq_summary.py $OUT/p${pn}_$kind$var > $OUT/sq${pn}_$kind$var.txt
    echo "== $arm pass $pn"; grep -E "kernel|vi_m|vi_march" $OUT/sq${pn}_$kind$var.txt
  done
done
