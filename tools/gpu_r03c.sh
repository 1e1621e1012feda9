#!/bin/bash
# round-3 session c (HEAD after the matrix-core transforms): the whole -m gpu suite, smoke(), the
# default bench line (C3 + its c3_100it / c3iso keys) and the BSD line.
# Each GPU step has its own time limit; a crash/abort/timeout ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03c
timeout -k 10 900 python -u -m pytest tests -q -m gpu -rfE --timeout 300 --timeout-method thread \
    > gpurun_out/r03c/gpu_tests.log 2>&1
rc=$?
echo "tests_exit=$rc"
tail -15 gpurun_out/r03c/gpu_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/r03c/smoke.log 2>&1 || { echo smoke_fail; tail -20 gpurun_out/r03c/smoke.log; exit 1; }
echo smoke_ok
timeout -k 10 400 python bench.py > gpurun_out/r03c/bench_c3.json 2> gpurun_out/r03c/bench_c3.err || { echo bench_fail; tail -20 gpurun_out/r03c/bench_c3.err; exit 1; }
cat gpurun_out/r03c/bench_c3.json
timeout -k 10 300 python bench.py --config bsd --no-cpu-baseline > gpurun_out/r03c/bench_bsd.json 2> gpurun_out/r03c/bench_bsd.err || { echo bsd_fail; tail -20 gpurun_out/r03c/bench_bsd.err; exit 1; }
cat gpurun_out/r03c/bench_bsd.json
exit $rc
