#!/bin/bash
# matrix-core column pass (csrc/gcol_mm.hpp): its GPU tests, the generic suite, then BSD A/B
# (ADMM_GCOL_MM=0: the LDS column pass) and a rocprof kernel summary of the BSD bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-mm}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_gcol_mm.py ${EXTRA_TESTS} -x -v -m gpu -rfE \
    --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo tests_fail; grep -E "FAIL|Error|error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for round in 1 2; do
  timeout -k 10 300 python3 tools/sweep.py --config bsd --steps 4 ADMM_GCOL_MM=0,1 ${SWEEP_KNOBS} >> $O/ab.txt 2>&1 || { echo sweep_fail; tail -20 $O/ab.txt; exit 1; }
done
cat $O/ab.txt
timeout -k 10 300 python bench.py --config bsd > $O/bench_bsd.json 2> $O/bench_bsd.err || { echo bench_fail; tail $O/bench_bsd.err; exit 1; }
cut -c1-400 $O/bench_bsd.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o run -- python3 bench.py --config bsd --no-cpu-baseline --no-parity --steps 3 > $O/prof.log 2>&1 || { echo prof_fail; tail $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_bsd.csv \;
echo mm_ok
