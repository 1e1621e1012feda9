#!/bin/bash
# SQ counters of the matrix-core column pass at the BSD size (one stream), three --pmc passes, each
# under its own time limit.  -> gpurun_out/sq_mm/{p1,p2,p3}
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/sq_mm"
mkdir -p "$OUT"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_INSTS_FLAT"
P3="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_WAVES"
i=0
for SET in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  ADMM_GEN_STREAMS=1 timeout -k 10 120 rocprofv3 --pmc $SET --kernel-include-regex "${KRE:-k_gcol_mm|k_grow}" --output-format csv -d "$OUT/p$i" -o run -- python3 tools/sweep.py --config bsd --steps 1 --maxit 10 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo sq_done
