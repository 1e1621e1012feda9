#!/bin/bash
# round-3 session d: the autograd files (second order through the native ops, op checks, concurrency).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03d
timeout -k 10 600 python -u -m pytest tests/test_gpu_second_order.py tests/test_gpu_ops.py tests/test_gpu_concurrency.py \
    tests/test_gpu_grad.py -v -s -m gpu -rfE --timeout 300 --timeout-method thread > gpurun_out/r03d/tests.log 2>&1
rc=$?
echo "tests_exit=$rc"
grep -E "PASS|FAIL|ERROR|passed|failed|aniso|iso_" gpurun_out/r03d/tests.log | tail -60
exit $rc
