#!/bin/bash
# tracer k-march: LLC parity, then LLC-90 benches (march default vs flat, KC sweep)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/trm; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_llc.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config llc90_synthetic --steps 20 --warmup 4 --no-cpu-baseline > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python -c "import json; d=json.load(open('$O/$name.json')); k=d['kernel_ms_mean']; print('%-14s step %.4f' % ('$name', d['ms_per_step']), {a: round(b*1e3,1) for a,b in k.items() if b}, d['thermo_overlap'])"
}
run at1s MGCM_THERMO_AT=1 MGCM_TRACER_PAIR=0 MGCM_TR_KC=5 MGCM_VI_KC=10 MGCM_MWG_EXCL=0
run at1s_x MGCM_THERMO_AT=1 MGCM_TRACER_PAIR=0 MGCM_TR_KC=5 MGCM_VI_KC=10
run at2s_x MGCM_THERMO_AT=2 MGCM_TRACER_PAIR=0 MGCM_TR_KC=5 MGCM_VI_KC=10
run at2p_x MGCM_THERMO_AT=2 MGCM_TR_KC=5 MGCM_VI_KC=10
run at2s MGCM_THERMO_AT=2 MGCM_TRACER_PAIR=0 MGCM_TR_KC=5 MGCM_VI_KC=10 MGCM_MWG_EXCL=0
run at2s_x_kc10 MGCM_THERMO_AT=2 MGCM_TRACER_PAIR=0 MGCM_TR_KC=10 MGCM_VI_KC=10
