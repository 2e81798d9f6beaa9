#!/bin/bash
# Round-1 GPU session: parity tests, smoke, bench, rocprofv3 kernel stats, HBM PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH_ARGS=${BENCH_ARGS:-"--steps 200 --warmup 20"}
timeout -k 10 600 python -m pytest tests -m gpu -q -s > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py $BENCH_ARGS --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { echo rocprof failed; tail -30 gpurun_out/prof.err; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_fetch.json 2> gpurun_out/pmc_fetch.err || { echo pmc fetch failed; tail -30 gpurun_out/pmc_fetch.err; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_write.json 2> gpurun_out/pmc_write.err || { echo pmc write failed; tail -30 gpurun_out/pmc_write.err; exit 1; }
ls -R gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write | grep -c csv
