#!/bin/bash
# round-3 final measurement session (after the pass B order / layout default change) (build of HEAD): whole -m gpu suite + smoke(), the default bench
# line (C3 + c3_100it / c3iso), the BSD line, a rocprofv3 kernel-stats run of the C3 bench, then the
# PMC request-size passes of this build (tools/pmc/run_rdreq.sh) and their summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03q
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -s -m gpu -rfE --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "tests_exit=$rc"
tail -4 $O/gpu_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { echo smoke_fail; tail -20 $O/smoke.log; exit 1; }
echo smoke_ok
timeout -k 10 400 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { echo bench_fail; tail -20 $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
timeout -k 10 300 python bench.py --config bsd --no-cpu-baseline > $O/bench_bsd.json 2> $O/bench_bsd.err || { echo bsd_fail; exit 1; }
cat $O/bench_bsd.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-extras > $O/prof.log 2>&1 || { echo prof_fail; exit 1; }
find $O/prof -name "*kernel_trace*" -delete
echo prof_ok
bash tools/pmc/run_rdreq.sh || exit 1
python3 tools/pmc/summarize_rdreq.py gpurun_out/rdreq $O/pmc_summary.json > $O/pmc.txt || exit 1
grep -E "pass_a|pass_b" $O/pmc.txt
exit $rc
