#!/bin/bash
# strip-height sweep of the training path (ADMM_PASSA_R: 0 = the library's rule) on C2, C3, C5 module
cd "$GRAFT_REPO_ROOT" || exit 1
for cfg in c2 c3 c5fwd; do
  for r in 0 4 8 16 0; do
    echo "== $cfg R=$r"
    ADMM_PASSA_R=$r timeout -k 10 120 python3 tools/bench_grad.py --config $cfg --maxit 20 --steps 3 2>/dev/null | tail -n 2 || exit 1
  done
done
