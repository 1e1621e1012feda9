#!/bin/bash
# A/B of library variants (tools/_variants/*.so) on the C3 and C2 sweeps; interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
for round in 1 2; do
  for v in tools/_variants/*.so; do
    echo "== $v round $round"
    ADMMTOR_LIB_OVERRIDE=$v timeout -k 10 200 python3 tools/sweep.py --config ${CFG:-c3} --steps 3 ${KNOBS} || exit 1
  done
done
