#!/bin/bash
# Round 6 final profiles (bench + rocprofv3 kernel stats + PMC passes per config), smoke, and
# the driver's own bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/r6j
mkdir -p $OUT
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo bench failed; tail -5 $OUT/bench_driver.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_driver.json')); c=d['cpu_baseline']; k=d['cs32x15']['cpu_baseline']; print('C2 20 steps', round(d['ms_per_step'],4), round(d['value'],1), 'cs32', round(d['cs32x15']['ms_per_step'],4), 'cpu', round(c['value'],1), round(c.get('all_cores',{}).get('value',0),1), c.get('all_cores',{}).get('tiling'), c.get('host_cpus_visible'), c.get('host_physical_cores'), 'cs32 cpu', round(k['value'],1), round(k.get('all_cores',{}).get('value',0),1), k.get('all_cores',{}).get('tiling'))"
bash profiles/run_r6.sh ocean90 cs32x15 llc90 > $OUT/prof.log 2>&1 || { echo profiles failed; tail -20 $OUT/prof.log; exit 1; }
grep -a '"ms_per_step"' $OUT/prof.log | head -0
for c in ocean90 cs32x15 llc90; do python3 -c "import json; d=json.load(open('gpurun_out/r6_$c/bench.json')); print('$c', round(d['ms_per_step'],4), round(d['value'],2), 'cpu', round(d['cpu_baseline']['value'],3), round(d['cpu_baseline'].get('all_cores',{}).get('value',0),3), d['cpu_baseline'].get('all_cores',{}).get('tiling'))"; done
