#!/bin/bash
# round-3 session h: the sharded files (2 and 8 ranks on cuda:0 over gloo), then the SQ counters of
# the C3 solve (pass A / pass B issue and LDS figures at HEAD).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03h
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -v -s -m gpu -rfE --timeout 500 --timeout-method thread \
    > gpurun_out/r03h/sharded.log 2>&1
rc=$?
echo "sharded_exit=$rc"
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r03h/sharded.log | tail -8
case $rc in 0|1) ;; *) exit $rc ;; esac
CFG=c3 bash tools/pmc/run_sq_cfg.sh || exit 1
python3 tools/pmc/summarize_sq.py gpurun_out/sq_c3 gpurun_out/r03h/sq_c3.json || exit 1
exit $rc
