#!/bin/bash
# PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs, per MI355X_MICROARCH.md) over
# the calibration kernels and the C3 bench; each step time-limited, chained with &&.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/calib_$C" -o run -- python3 tools/pmc/calib.py > "$OUT/calib_$C.log" 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/bench_$C" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity > "$OUT/bench_$C.log" 2>&1 || exit 1
done
echo pmc_ok
