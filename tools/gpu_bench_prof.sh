#!/bin/bash
# One measurement session: optional mimic sweep, the default bench (C3), a rocprofv3 kernel-stats
# run of the same command. Each GPU step has its own time limit; a failing step ends the script.
# Usage: TAG=r02a [MIMIC=MIXED_SWEEP] bash tools/gpu_bench_prof.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-run}
mkdir -p gpurun_out/$TAG
if [ -n "$MIMIC" ]; then
  env $MIMIC=1 timeout -k 10 300 tools/membench/stream_mimic > gpurun_out/$TAG/mimic.txt 2>&1 || { echo mimic_fail; exit 1; }
  echo mimic_ok
fi
timeout -k 10 300 python bench.py $BENCH_ARGS > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo bench_fail; tail gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/prof" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity $BENCH_ARGS > gpurun_out/$TAG/prof.log 2>&1 || { echo prof_fail; exit 1; }
find gpurun_out/$TAG/prof -name "*kernel_trace*" -delete
echo prof_ok
