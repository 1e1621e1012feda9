#!/bin/bash
# SQ counters of the library variants in tools/_variants (one rocprofv3 pass each, C3, 10 iterations)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/sqv"
mkdir -p "$OUT"
SET=${SET:-"SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS"}
for v in tools/_variants/*.so; do
  n=$(basename $v .so)
  ADMMTOR_LIB_OVERRIDE=$v timeout -k 10 240 rocprofv3 --pmc $SET --output-format csv -d "$OUT/$n" -o run -- python3 tools/sweep.py --config ${CFG:-c3} --steps 1 --maxit 10 > "$OUT/$n.log" 2>&1 || { echo "$n failed"; tail -5 "$OUT/$n.log"; exit 1; }
done
echo sqv_done
