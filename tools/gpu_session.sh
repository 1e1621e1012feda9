#!/bin/bash
# One GPU session on the box: pytest -m gpu (whole suite, or a -k selection), smoke(), the default bench
# line, and a rocprofv3 kernel-trace summary of the same bench.  Every GPU step has its own time limit; a
# crash / abort / timeout ends the session.  Results under gpurun_out/<tag>/.
# usage (through gpurun): bash tools/gpu_session.sh <tag> [pytest -k expression | all | none] [bench|nobench]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-session}
SEL=${2:-all}
BENCH=${3:-bench}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ "$SEL" != "none" ]; then
    if [ "$SEL" = "all" ]; then K=(); else K=(-k "$SEL"); fi
    timeout -k 10 1500 python -u -m pytest tests -q -m gpu -rfE -s --timeout 300 --timeout-method thread "${K[@]}" \
        > "$OUT/tests.log" 2>&1
    rc=$?
    echo "tests_exit=$rc"
    tail -25 "$OUT/tests.log"
    case $rc in 0|1|5) ;; *) exit $rc ;; esac
    timeout -k 10 300 python -u __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || { echo smoke_fail; tail -20 "$OUT/smoke.log"; exit 1; }
    echo smoke_ok
fi
if [ "$BENCH" = "bench" ]; then
    timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo bench_fail; tail -20 "$OUT/bench.err"; exit 1; }
    echo bench_ok
    head -c 3000 "$OUT/bench.json"; echo
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o prof -- python3 bench.py --steps 5 --warmup 2 \
        --no-cpu-baseline > "$OUT/bench_rocprof.json" 2> "$OUT/bench_rocprof.err" || { echo rocprof_fail; tail -20 "$OUT/bench_rocprof.err"; exit 1; }
    echo rocprof_ok
fi
exit ${rc:-0}
