#!/bin/bash
# Run GPU steps given as arguments in order, each under its own time limit, stopping at the first failure.
# Step syntax:  "NAME:SECONDS:command ..."  -> output in gpurun_out/steps/NAME.log, tail printed.
# usage (through gpurun): bash tools/gpu_steps.sh "tests:600:python -u -m pytest tests/x.py -q" "bench:300:python bench.py"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/steps
for step in "$@"; do
  name=${step%%:*}; rest=${step#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/steps/$name.log" 2>&1
  rc=$?
  grep -v "amdgpu.ids\|socket.cpp" "gpurun_out/steps/$name.log" | tail -${TAILN:-12}
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
