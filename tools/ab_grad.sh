#!/bin/bash
# A/B of library variants (tools/_variants/*.so) on the training path (tools/bench_grad.py).
cd "$GRAFT_REPO_ROOT" || exit 1
for v in tools/_variants/*.so; do
  for cfg in "c3 --maxit 20" "c5fwd"; do
    for ppg in ${PPGS:-8}; do
      echo "== $v $cfg ppg=$ppg"
      ADMM_ISO_PPG=$ppg ADMMTOR_LIB_OVERRIDE=$v timeout -k 10 200 python3 tools/bench_grad.py --config $cfg || exit 1
    done
  done
done
