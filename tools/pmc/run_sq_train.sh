#!/bin/bash
# SQ counters of the training path at the C5 module shape (tools/bench_grad.py --config c5fwd: forward with
# history + native backward, 20 iterations), two --pmc passes, each under its own time limit, restricted
# to the backward and forward row / column kernels.  -> gpurun_out/sq_train/{p1,p2}
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/sq_train"
mkdir -p "$OUT"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_INSTS_FLAT"
i=0
for SET in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -k 10 180 rocprofv3 --pmc $SET --kernel-include-regex "k_bwd|k_pass|k_iso" --output-format csv -d "$OUT/p$i" -o run -- python3 tools/bench_grad.py --config c5fwd --steps 1 --maxit 20 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo sq_done
