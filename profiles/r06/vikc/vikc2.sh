#!/bin/bash
# Round 6: k_mom_vi_m2 over whole columns (one chunk) as LLC-90's default -- parity (LLC-30 VI
# forms incl. ragged 3-level chunks, LLC-90 full size), A/B against two chunks (MGCM_VI_KC=25)
# alternating, then the LLC-90 profile at HEAD (profiles/run_r6.sh llc90).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${1:-r6v}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_llc.py -m gpu -x -v -s -k "vi or full_size" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -a "FAILED\|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2 3; do
  for kc in 0 25; do
    if [ $kc = 0 ]; then unset MGCM_VI_KC; else export MGCM_VI_KC=$kc; fi
    timeout -k 10 200 python3 bench.py --config llc90_synthetic --steps 40 --warmup 6 --no-cpu-baseline --no-cs32 > $OUT/llc_kc${kc}_$rep.json 2> $OUT/llc_kc${kc}_$rep.err || { echo bench failed; tail -5 $OUT/llc_kc${kc}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/llc_kc${kc}_$rep.json')); print('LLC kc=$kc', round(d['ms_per_step'],4), 'mom', round(d['kernel_ms_mean']['mom_step']*1e3,1))"
  done
done
unset MGCM_VI_KC
bash profiles/run_r6.sh llc90 > $OUT/prof.log 2>&1 || { echo prof failed; tail -20 $OUT/prof.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6_llc90/bench.json')); print('llc90 prof', round(d['ms_per_step'],4), round(d['value'],2))"
