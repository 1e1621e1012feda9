#!/bin/bash
# A mixed-kernel variant (tools/_variants/<name>.so) on the GPU: the mixed-path tests on it, then interleaved
# A/B against the default library on each given bench config (tools/gpu_ab_mixed.sh).
# usage: bash tools/gpu_ab_variant.sh <name> <config> [<config> ...]   -> gpurun_out/ab_<config>.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
V=$1; shift
ADMMTOR_LIB_OVERRIDE=tools/_variants/$V.so timeout -k 10 600 python -u -m pytest tests/test_gpu_mixed.py -q -x \
  --timeout 300 --timeout-method thread > gpurun_out/mixed_$V.log 2>&1 || { echo "mixed tests failed: $V"; tail -5 gpurun_out/mixed_$V.log; exit 1; }
echo "mixed tests ok: $V"
for cfg in "$@"; do
  bash tools/gpu_ab_mixed.sh "$cfg" "$V" > /dev/null || exit 1
done
echo ab_done
