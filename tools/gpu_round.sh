#!/bin/bash
# one GPU session: tests, bench (C3 default + C3 at 100 it + C2), rocprof kernel stats, PMC traffic.
# Each GPU step has its own time limit; a failing step ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu -s > gpurun_out/gpu_tests.log 2>&1
echo "tests_exit=$?"
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench_fail; exit 1; }
timeout -k 10 300 python bench.py --config c3x100 --steps 5 --no-cpu-baseline > gpurun_out/bench_c3x100.json 2>> gpurun_out/bench.err || { echo bench100_fail; exit 1; }
timeout -k 10 300 python bench.py --config c2 --steps 20 --no-cpu-baseline > gpurun_out/bench_c2.json 2>> gpurun_out/bench.err || { echo benchc2_fail; exit 1; }
echo "bench_ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/prof.log 2>&1 || { echo prof_fail; exit 1; }
find gpurun_out/prof -name "*kernel_trace*" -delete
echo "prof_ok"
if [ -n "$WITH_PMC" ]; then bash tools/pmc/run_pmc.sh || exit 1; fi
