#!/bin/bash
# block shapes of the generic path under the two-stream solve (BSD bench)
cd "$GRAFT_REPO_ROOT" || exit 1
for c in 2 4 8; do for l in 1 2 4; do
  echo "== cols=$c lines=$l"
  ADMM_GCOL_COLS=$c ADMM_GROW_LINES=$l timeout -k 10 100 python3 bench.py --config bsd --steps 10 --no-cpu-baseline --no-parity | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['value'],1))" || exit 1
done; done
