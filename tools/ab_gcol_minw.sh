#!/bin/bash
# A/B: column-pass occupancy hint (tools/_variants/{base,w4}.so) x columns per block, BSD bench
cd "$GRAFT_REPO_ROOT" || exit 1
for round in 1 2; do
  for v in base w4; do for c in 2 4; do
    echo "== $v cols=$c round $round"
    ADMM_GCOL_COLS=$c ADMMTOR_LIB_OVERRIDE=tools/_variants/$v.so timeout -k 10 200 python3 bench.py --config bsd --steps 5 --no-cpu-baseline --no-parity | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['roofline']['per_kernel']['pass_b']['ms_total']/d['roofline']['per_kernel']['pass_b']['launches'],4))" || exit 1
  done; done
done
