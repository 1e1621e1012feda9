#!/bin/bash
# HBM bytes from the memory-side request-size counters (no calibration factor needed):
#   read  = 32 n32 + 64 n64 + 128 n128  (TCC_EA0_RDREQ_{32B,64B,128B}; their sum is TCC_EA0_RDREQ)
#   write = 64 n64 + 32 (n - n64)        (TCC_EA0_WRREQ, TCC_EA0_WRREQ_64B)
# over the calibration kernels (known bytes) and the C3 bench; one rocprofv3 pass per counter set.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/rdreq"
mkdir -p "$OUT"
# the build the counters belong to (bench.py reports traffic only from a summary of its own build)
python3 -c "import sys; sys.path.insert(0, 'torch-admm-deconv_amd'); from admmtor import _native; print(_native.load().admm_tv_build_hash().decode())" > "$OUT/build_hash.txt" || exit 1
RD="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
WR="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
i=0
for SET in "$RD" "$WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d "$OUT/calib$i" -o run -- python3 tools/pmc/calib.py > "$OUT/calib$i.log" 2>&1 || { echo "calib pass $i failed"; tail -3 "$OUT/calib$i.log"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc $SET --output-format csv -d "$OUT/bench$i" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-extras > "$OUT/bench$i.log" 2>&1 || { echo "bench pass $i failed"; tail -3 "$OUT/bench$i.log"; exit 1; }
done
echo rdreq_done
