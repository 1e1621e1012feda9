#!/bin/bash
# A mixed-kernel variant (tools/_variants/<name>.so) on the GPU: the mixed-path tests on it, then the HD
# A/B against the default library (tools/gpu_ab_mixed.sh).  usage: bash tools/gpu_ab_variant_hd.sh <name>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
ADMMTOR_LIB_OVERRIDE=tools/_variants/$1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_mixed.py -q -x \
  --timeout 300 --timeout-method thread > gpurun_out/mixed_$1.log 2>&1 || { echo "mixed tests failed: $1"; tail -5 gpurun_out/mixed_$1.log; exit 1; }
echo "mixed tests ok: $1"
bash tools/gpu_ab_mixed.sh hd "$1"
