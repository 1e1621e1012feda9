#!/bin/bash
# one GPU session: tests, bench, rocprof kernel stats.  Each GPU step has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu -s > gpurun_out/gpu_tests.log 2>&1
echo "tests_exit=$?"
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench_fail; exit 1; }
echo "bench_exit=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/prof.log 2>&1
echo "prof_exit=$?"
