#!/bin/bash
# (historical: the device-function body and MGCM_VI_LBW were removed after this A/B -- slower)
# Round 6: k_mom_vi_m2's body as a device function (189 VGPRs at 2 waves per SIMD; capped for 3
# waves per SIMD: 168 VGPRs with 20 spilled, MGCM_VI_LBW=3) against the inline kernel of the
# committed library (215 VGPRs; _variants/lib_vi_orig.so): LLC-30 parity of both new forms,
# LLC-90 alternating, rocprofv3 kernel time of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6w3}
mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || MGCM_VI_LBW=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_llc.py -m gpu -x -v -s --timeout 200 --timeout-method thread -k "vi or None or full_size" > $OUT/pytest3.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error" $OUT/pytest3.log | head; tail -30 $OUT/pytest3.log; exit 1; }
tail -1 $OUT/pytest3.log
for rep in 1 2; do
  for v in orig b2 b3; do
    case $v in orig) E="MGCM_LIB=$PWD/mitgcm_amd/_build/diag/lib_vi_orig.so" ;; b2) E="MGCM_VI_LBW=2" ;; b3) E="MGCM_VI_LBW=3" ;; esac
    env $E timeout -k 10 200 python3 bench.py --config llc90_synthetic --steps 40 --warmup 6 --no-cpu-baseline --no-cs32 > $OUT/llc_${v}_$rep.json 2> $OUT/llc_${v}_$rep.err || { echo bench failed; tail -5 $OUT/llc_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/llc_${v}_$rep.json')); k=d['kernel_ms_mean']; print('LLC $v', round(d['ms_per_step'],4), 'mom_step ms', round(k['mom_step'],4))"
  done
done
for v in orig b2 b3; do
  case $v in orig) E="MGCM_LIB=$PWD/mitgcm_amd/_build/diag/lib_vi_orig.so" ;; b2) E="MGCM_VI_LBW=2" ;; b3) E="MGCM_VI_LBW=3" ;; esac
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python3 bench.py --config llc90_synthetic --steps 30 --warmup 4 --no-cpu-baseline --no-cs32 > $OUT/prof_$v.json 2> $OUT/prof_$v.err || { echo rocprof failed; tail -5 $OUT/prof_$v.err; exit 1; }
  f=$(find $OUT/prof_$v -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'vi_m2' in r['Name']: print('$v', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
done
