#!/bin/bash
# round-3 session: the whole GPU suite + smoke, the default bench (C3 with the C3-100 and C3-iso
# extras), the BSD bench, a rocprofv3 kernel-stats run of the default bench, the PMC traffic passes.
# Each GPU step has its own time limit; a crash / timeout ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-r03a}
mkdir -p gpurun_out/$T
bash tools/gpu_tests.sh; rc=$?
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo bench_fail; tail gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json
timeout -k 10 300 python bench.py --config bsd --steps 20 --no-cpu-baseline > gpurun_out/$T/bench_bsd.json 2>> gpurun_out/$T/bench.err || { echo bsd_fail; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$T/prof" -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/$T/prof.log 2>&1 || { echo prof_fail; exit 1; }
find gpurun_out/$T/prof -name "*kernel_trace*" -delete
echo prof_ok
if [ -n "$WITH_PMC" ]; then bash tools/pmc/run_rdreq.sh || exit 1; fi
exit $rc
