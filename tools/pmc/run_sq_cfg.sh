#!/bin/bash
# SQ counters of one bench config (two rocprofv3 --pmc passes, each under its own time limit).
# Usage: CFG=bsd bash tools/pmc/run_sq_cfg.sh   -> gpurun_out/sq_$CFG/{p1,p2}
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
CFG=${CFG:-bsd}
OUT="$GRAFT_REPO_ROOT/gpurun_out/sq_$CFG"
mkdir -p "$OUT"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_INSTS_FLAT"
i=0
for SET in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -k 10 120 rocprofv3 --pmc $SET --output-format csv -d "$OUT/p$i" -o run -- python3 tools/sweep.py --config $CFG --steps 1 --maxit 10 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo sq_done
