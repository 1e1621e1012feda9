#!/bin/bash
# Interleaved A/B of the mixed-radix kernel variants (tools/build_mixed_variant.sh) on one box:
# tools/sweep.py on a config for the default library and each variant, two rounds.
# usage: bash tools/gpu_ab_mixed.sh <config> <variant> [<variant> ...]   -> gpurun_out/ab_<config>.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
CFG=$1; shift
OUT=gpurun_out/ab_$CFG.txt
mkdir -p gpurun_out
: > "$OUT"
for round in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then LIB=""; else LIB="tools/_variants/$v.so"; fi
    echo "round $round variant $v" >> "$OUT"
    ADMMTOR_LIB_OVERRIDE=$LIB timeout -k 10 180 python tools/sweep.py --config "$CFG" --steps 5 >> "$OUT" 2>&1 || { echo "sweep failed: $v"; tail -5 "$OUT"; exit 1; }
  done
done
cat "$OUT"
