#!/bin/bash
# channel-statistics tests + bench, the C5 training step with the HIP ChannelPool (and, unless
# SKIP_C5_TORCH, with PyTorch's), and (WITH_PROF) a rocprofv3 kernel-stats run of the C5 step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chanpool.py -x -v --timeout 120 --timeout-method thread > gpurun_out/chanpool_tests.log 2>&1 || { echo tests_fail; exit 1; }
timeout -k 10 200 python -u tools/bench_chanpool.py > gpurun_out/chanpool_bench.txt 2>&1 || { echo cbench_fail; exit 1; }
[ -n "$SKIP_C5" ] && exit 0
timeout -k 10 600 python -u bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/c5_native.json 2> gpurun_out/c5_native.err || { echo c5n_fail; exit 1; }
if [ -z "$SKIP_C5_TORCH" ]; then
  ADMMTOR_CHANPOOL=torch timeout -k 10 600 python -u bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/c5_torch.json 2> gpurun_out/c5_torch.err || { echo c5t_fail; exit 1; }
fi
if [ -n "$WITH_PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_c5" -o run -- python3 -u bench.py --config c5 --steps 1 --warmup 1 > gpurun_out/prof_c5.log 2>&1 || { echo prof_fail; exit 1; }
  find gpurun_out/prof_c5 -name "*kernel_trace*" -delete
fi
echo done
