#!/bin/bash
# iso plane-group size A/B (ADMM_ISO_PPG; 0 = the library's rule): inference sweep and training path at C3 iso
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 python3 tools/sweep.py --config c3iso --steps 3 ADMM_ISO_PPG=0,16,0,16 || exit 1
for p in 0 16 0 16; do
  echo "== ppg=$p"
  ADMM_ISO_PPG=$p timeout -k 10 200 python3 tools/bench_grad.py --config c3iso --maxit 20 --steps 3 2>/dev/null | tail -n 1 || exit 1
done
