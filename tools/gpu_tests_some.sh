#!/bin/bash
# GPU test subset: TESTS="tests/a.py tests/b.py" bash tools/gpu_tests_some.sh  (no -x; each file reports)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest $TESTS -q -m gpu -rfE -s --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_some.log 2>&1
rc=$?
echo "tests_exit=$rc"
tail -40 gpurun_out/gpu_tests_some.log
exit $rc
