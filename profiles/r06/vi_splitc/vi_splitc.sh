#!/bin/bash
# (historical: the MGCM_VI_SPLITC form was removed after this A/B -- slower)
# Round 6: k_mom_vi_m2 with one component per workgroup (MGCM_VI_SPLITC=1: 168 VGPRs, 3 waves
# per SIMD) against both components per workgroup (189 VGPRs, 2 waves): parity (LLC-30 every
# form, LLC-90 full size), then LLC-90 alternating, then rocprofv3 kernel stats of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6v1}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_llc.py -m gpu -x -v -s --timeout 200 --timeout-method thread -k "vi or None or full_size" > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for sc in 0 1; do
    MGCM_VI_SPLITC=$sc timeout -k 10 200 python3 bench.py --config llc90_synthetic --steps 40 --warmup 6 --no-cpu-baseline --no-cs32 > $OUT/llc_sc${sc}_$rep.json 2> $OUT/llc_sc${sc}_$rep.err || { echo bench failed; tail -5 $OUT/llc_sc${sc}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/llc_sc${sc}_$rep.json')); k=d['kernel_ms_mean']; print('LLC sc=$sc', round(d['ms_per_step'],4), 'mom_step ms', round(k['mom_step'],4))"
  done
done
for sc in 0 1; do
  MGCM_VI_SPLITC=$sc timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof$sc -o run --output-format csv -- python3 bench.py --config llc90_synthetic --steps 30 --warmup 4 --no-cpu-baseline --no-cs32 > $OUT/prof$sc.json 2> $OUT/prof$sc.err || { echo rocprof failed; tail -5 $OUT/prof$sc.err; exit 1; }
  f=$(find $OUT/prof$sc -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'vi_m2' in r['Name']: print('sc=$sc', r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
done
