#!/bin/bash
# round-3 session b: the 2-rank multi-GPU rehearsal of bench.py (both ranks on cuda:0 over gloo,
# ADMM_BENCH_REHEARSAL=1; the driver's N > 1 runs use RCCL on a node), then the SQ counters of the
# generic path at the BSD size.  Each GPU step has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03b
timeout -k 10 300 python -u -m pytest tests/test_gpu_concurrency.py tests/test_gpu_generic.py -q -m gpu -rfE \
    --timeout 200 --timeout-method thread > gpurun_out/r03b/tests.log 2>&1 || { echo tests_fail; tail -20 gpurun_out/r03b/tests.log; exit 1; }
tail -2 gpurun_out/r03b/tests.log
ADMM_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 4 --warmup 1 \
    > gpurun_out/r03b/bench_rehearsal_n2.json 2> gpurun_out/r03b/bench_rehearsal_n2.err || { echo rehearsal_fail; tail -20 gpurun_out/r03b/bench_rehearsal_n2.err; exit 1; }
cat gpurun_out/r03b/bench_rehearsal_n2.json
CFG=bsd bash tools/pmc/run_sq_cfg.sh || exit 1
# generic path: solves on 1-4 streams (ADMM_GEN_STREAMS), BSD / VGA / HD, interleaved rounds
for round in 1 2; do
  for cfg in bsd; do
    timeout -k 10 200 python3 tools/sweep.py --config $cfg --steps 4 ADMM_GEN_STREAMS=1,2,3,4 >> gpurun_out/r03b/gen_streams.txt 2>&1 || exit 1
  done
done
echo streams_ok
