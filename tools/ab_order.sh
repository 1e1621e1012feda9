#!/bin/bash
# pass order A/B: pass B block remap / plane order (ADMM_PASSB_PMODE) x pass A strip order
# (ADMM_PASSA_REV) x pass B plane groups (ADMM_PASSB_GP), C3 (CFG), interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for round in 1 2; do
  echo "== round $round"
  timeout -k 10 300 python3 tools/sweep.py --config ${CFG:-c3} --steps 3 ADMM_PASSB_PMODE=${PM:-2,3,4,5} ADMM_PASSA_REV=${AR:-0,1} ADMM_PASSB_GP=${GPS:-1} || exit 1
done
