#!/bin/bash
# round-3 records at the final build: BSD kernel stats (rocprofv3), C2 line, 2-rank bench rehearsal
# (both ranks on cuda:0 over gloo, ADMM_BENCH_REHEARSAL=1; the driver's N > 1 runs use RCCL).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof_bsd" -o run -- python3 bench.py --config bsd --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/prof_bsd.log 2>&1 || { echo prof_fail; exit 1; }
find $O/prof_bsd -name "*kernel_trace*" -delete
echo prof_ok
timeout -k 10 300 python bench.py --config c2 --steps 20 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { echo c2_fail; exit 1; }
cat $O/bench_c2.json
ADMM_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 4 --warmup 1 \
    > $O/bench_rehearsal_n2.json 2> $O/bench_rehearsal_n2.err || { echo rehearsal_fail; tail -20 $O/bench_rehearsal_n2.err; exit 1; }
cat $O/bench_rehearsal_n2.json
