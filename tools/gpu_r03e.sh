#!/bin/bash
# round-3 session e: the autograd GPU files (second order through the native ops) and the column-strip
# layout mimic (pass A / pass B access patterns without FFT work, tools/membench STRIP_SWEEP).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03e
STRIP_SWEEP=1 timeout -k 10 120 ./tools/membench/stream_mimic > gpurun_out/r03e/strip_sweep.txt 2>&1 || { echo mimic_fail; cat gpurun_out/r03e/strip_sweep.txt; exit 1; }
cat gpurun_out/r03e/strip_sweep.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_second_order.py tests/test_gpu_ops.py tests/test_gpu_concurrency.py \
    tests/test_gpu_grad.py -v -s -m gpu -rfE --timeout 300 --timeout-method thread > gpurun_out/r03e/tests.log 2>&1
rc=$?
echo "tests_exit=$rc"
grep -E "PASS|FAIL|ERROR|passed|failed|aniso|iso_" gpurun_out/r03e/tests.log | tail -60
exit $rc
