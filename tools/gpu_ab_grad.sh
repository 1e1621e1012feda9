#!/bin/bash
# Interleaved A/B of library variants on the training path (tools/bench_grad.py --config c5fwd, the C5
# module shape), two rounds, each run under its own time limit, plus the gradient tests on each variant.
# usage: bash tools/gpu_ab_grad.sh <variant> [<variant> ...]   -> gpurun_out/ab_grad.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/ab_grad.txt
mkdir -p gpurun_out
: > "$OUT"
for v in "$@"; do
  ADMMTOR_LIB_OVERRIDE=tools/_variants/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_grad.py -q -x \
    --timeout 300 --timeout-method thread > gpurun_out/grad_tests_$v.log 2>&1 || { echo "grad tests failed: $v"; tail -5 gpurun_out/grad_tests_$v.log; exit 1; }
  echo "grad tests ok: $v"
done
for round in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then LIB=""; else LIB="tools/_variants/$v.so"; fi
    echo "round $round variant $v" >> "$OUT"
    ADMMTOR_LIB_OVERRIDE=$LIB timeout -k 10 200 python tools/bench_grad.py --config c5fwd --steps 3 >> "$OUT" 2>&1 || { echo "bench_grad failed: $v"; exit 1; }
  done
done
cat "$OUT"
