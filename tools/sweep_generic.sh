cd "$GRAFT_REPO_ROOT" || exit 1
for c in 2 4 8 16; do for l in 1 2 4; do
  echo "== cols=$c lines=$l"
  ADMM_GCOL_COLS=$c ADMM_GROW_LINES=$l timeout -k 10 100 python3 bench.py --config bsd --steps 5 --no-cpu-baseline --no-parity || exit 1
done; done
