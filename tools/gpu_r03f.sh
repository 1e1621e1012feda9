#!/bin/bash
# round-3 session f: whole -m gpu suite + smoke() at HEAD, then the PMC request-size passes of the C3
# bench on this build (tools/pmc/run_rdreq.sh), so the round-end bench line resolves its traffic.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03f
timeout -k 10 900 python -u -m pytest tests -q -s -m gpu -rfE --timeout 300 --timeout-method thread \
    > gpurun_out/r03f/gpu_tests.log 2>&1
rc=$?
echo "tests_exit=$rc"
tail -8 gpurun_out/r03f/gpu_tests.log
grep -E "bf16 autocast" gpurun_out/r03f/gpu_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/r03f/smoke.log 2>&1 || { echo smoke_fail; tail -20 gpurun_out/r03f/smoke.log; exit 1; }
echo smoke_ok
bash tools/pmc/run_rdreq.sh || exit 1
python3 tools/pmc/summarize_rdreq.py gpurun_out/rdreq gpurun_out/r03f/pmc_summary.json || exit 1
exit $rc
