#!/bin/bash
# channel-statistics tests + bench, and the C5 training step with the HIP ChannelPool vs PyTorch's
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chanpool.py -x -v --timeout 120 --timeout-method thread > gpurun_out/chanpool_tests.log 2>&1 || { echo tests_fail; exit 1; }
timeout -k 10 200 python -u tools/bench_chanpool.py > gpurun_out/chanpool_bench.txt 2>&1 || { echo cbench_fail; exit 1; }
[ -n "$SKIP_C5" ] && exit 0
timeout -k 10 600 python -u bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/c5_native.json 2> gpurun_out/c5_native.err || { echo c5n_fail; exit 1; }
[ -n "$SKIP_C5_TORCH" ] && exit 0
ADMMTOR_CHANPOOL=torch timeout -k 10 600 python -u bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/c5_torch.json 2> gpurun_out/c5_torch.err || { echo c5t_fail; exit 1; }
echo done
