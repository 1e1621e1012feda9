#!/bin/bash
# Column-schedule variant (tools/_variants/mcolv.so): mixed-path tests on it, then interleaved A/B against the
# default library on the 4K UHD and 360x720 workloads.  -> gpurun_out/ab_uhd.txt, gpurun_out/ab_sd.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
ADMMTOR_LIB_OVERRIDE=tools/_variants/mcolv.so timeout -k 10 600 python -u -m pytest tests/test_gpu_mixed.py -q -x \
  --timeout 300 --timeout-method thread > gpurun_out/mixed_mcolv.log 2>&1 || { echo "mixed tests failed"; tail -5 gpurun_out/mixed_mcolv.log; exit 1; }
echo mixed_tests_ok
bash tools/gpu_ab_mixed.sh uhd mcolv > /dev/null && bash tools/gpu_ab_mixed.sh sd mcolv > /dev/null && echo ab_done
