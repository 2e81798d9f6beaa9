#!/bin/bash
# SQ counter pass over a short bench run (one --pmc pass, <= 8 SQ counters), summarised per
# kernel by tools/sq_summary.py.   CONFIG=llc90_synthetic OUT=gpurun_out/sq
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
CONFIG=${CONFIG:-llc90_synthetic}
OUT=${OUT:-gpurun_out/sq}
mkdir -p $OUT
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $OUT/pmc -o run --output-format csv -- python3 bench.py --config $CONFIG --steps 6 --warmup 1 --no-cpu-baseline > $OUT/bench.json 2> $OUT/pmc.err || { echo pmc failed; grep -v "^[EW]2026" $OUT/pmc.err | tail -20; exit 1; }
python tools/sq_summary.py $OUT/pmc > $OUT/sq_summary.txt && cat $OUT/sq_summary.txt
