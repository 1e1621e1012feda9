#!/bin/bash
# A/B: generic aniso inference on one stream vs two plane halves on two streams (ADMM_GEN_STREAMS)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
ADMM_GEN_STREAMS=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_generic.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/gen_streams_tests.log 2>&1 || { echo tests_fail; tail -20 gpurun_out/gen_streams_tests.log; exit 1; }
tail -1 gpurun_out/gen_streams_tests.log
for round in 1 2; do
  for n in 1 2; do
    echo "== streams=$n round $round"
    ADMM_GEN_STREAMS=$n timeout -k 10 200 python3 bench.py --config bsd --steps 10 --no-cpu-baseline --no-parity | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1))" || exit 1
  done
done
for n in 1 2; do echo "== sizes streams=$n"; ADMM_GEN_STREAMS=$n timeout -k 10 300 python3 tools/bench_generic_sizes.py 2>&1 | grep -v amdgpu.ids || exit 1; done
