#!/bin/bash
# GPU test session: the whole -m gpu suite (no -x: every file reports), then smoke().
# Each GPU step has its own time limit; a crash/abort/timeout ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -rfE -s --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "tests_exit=$rc"
tail -30 gpurun_out/gpu_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo smoke_fail; tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke_ok
exit $rc
