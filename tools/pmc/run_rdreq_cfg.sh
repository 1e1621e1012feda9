#!/bin/bash
# HBM bytes per kernel (memory-side request-size counters, as run_rdreq.sh) for one bench config
# (bsd, hd, c2, ...), one stream (ADMM_GEN_STREAMS=1), 1 step + 1 warm-up, plus the calibration copies.
# usage: bash tools/pmc/run_rdreq_cfg.sh <config> [tag]   -> gpurun_out/rdreq_<config>[_<tag>]/
# (A/B knobs: run it with ADMMTOR_LIB_OVERRIDE=<the A/B library> and the knob in the environment)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
CFG=${1:-bsd}
OUT="$GRAFT_REPO_ROOT/gpurun_out/rdreq_$CFG${2:+_$2}"
mkdir -p "$OUT"
python3 -c "import sys; sys.path.insert(0, 'torch-admm-deconv_amd'); from admmtor import _native; print(_native.load().admm_tv_build_hash().decode())" > "$OUT/build_hash.txt" || exit 1
RD="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
WR="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
i=0
for SET in "$RD" "$WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d "$OUT/calib$i" -o run -- python3 tools/pmc/calib.py > "$OUT/calib$i.log" 2>&1 || { echo "calib pass $i failed"; tail -3 "$OUT/calib$i.log"; exit 1; }
  ADMM_GEN_STREAMS=1 timeout -s KILL 240 rocprofv3 --pmc $SET --output-format csv -d "$OUT/bench$i" -o run -- python3 bench.py --config "$CFG" --steps 1 --warmup 1 --no-cpu-baseline --no-parity --no-extras > "$OUT/bench$i.log" 2>&1 || { echo "bench pass $i failed"; tail -3 "$OUT/bench$i.log"; exit 1; }
done
echo rdreq_done
