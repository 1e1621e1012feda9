#!/bin/bash
# A/B of library variants (tools/_variants/*.so) on the generic-size bench (bench.py --config bsd)
cd "$GRAFT_REPO_ROOT" || exit 1
for round in 1 2; do
  for v in tools/_variants/*.so; do
    echo "== $v round $round"
    ADMMTOR_LIB_OVERRIDE=$v timeout -k 10 200 python3 bench.py --config ${CFG:-bsd} --steps 5 --no-cpu-baseline --no-parity || exit 1
  done
done
