#!/bin/bash
# Round-4 final measurements: the LLC / latlon parity tests, then rocprof + PMC profiles of
# the three configs (profiles/run_r4.sh), then the sharded N=1 RCCL bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_final
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_llc.py tests/test_gpu_ocean90.py tests/test_gpu_refhost.py > gpurun_out/r4_final/pytest.log 2>&1 || { echo pytest failed; tail -20 gpurun_out/r4_final/pytest.log; exit 1; }
tail -1 gpurun_out/r4_final/pytest.log
bash profiles/run_r4.sh ocean90 llc90 cs32x15 || exit 1
NOTEST=1 CONFIGS="llc90_synthetic global_ocean.cs32x15" TAG=r4_final/shard bash tools/shard_check.sh || exit 1
