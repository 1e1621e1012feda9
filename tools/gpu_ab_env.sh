#!/bin/bash
# Interleaved A/B of environment knobs on one bench config: bench.py --config <cfg> for each setting, two
# rounds, each run under its own time limit; the bench's JSON line (value, roofline) per run.  The knobs are
# read only by the A/B build of the library (csrc/knobs.hpp), which this script loads
# (admmtor/_lib/libadmm_tv_ab.so, built by the Makefile) unless ADMMTOR_LIB_OVERRIDE is set.
# usage: bash tools/gpu_ab_env.sh <config> "A=1 B=2" "A=0 B=2" ...   -> gpurun_out/ab_env_<config>.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
export ADMMTOR_LIB_OVERRIDE=${ADMMTOR_LIB_OVERRIDE:-$GRAFT_REPO_ROOT/torch-admm-deconv_amd/admmtor/_lib/libadmm_tv_ab.so}
CFG=$1; shift
OUT=gpurun_out/ab_env_$CFG.txt
mkdir -p gpurun_out
: > "$OUT"
for round in 1 2; do
  for setting in "$@"; do
    echo "round $round: $setting" >> "$OUT"
    env $setting timeout -k 10 240 python3 bench.py --config "$CFG" --steps 10 --warmup 2 --no-cpu-baseline --no-extras \
      --no-parity >> "$OUT" 2>/dev/null || { echo "bench failed: $setting"; exit 1; }
  done
done
python3 - "$OUT" <<'EOF'
import json, sys
lines = open(sys.argv[1]).read().splitlines()
for i, l in enumerate(lines):
    if l.startswith("round"):
        tag = l
    elif l.startswith("{"):
        d = json.loads(l)
        per = d["roofline"].get("per_kernel", {})
        print(f"{tag:60s} {d['value']:9.1f} it/s  " + "  ".join(f"{k} {v['ms_total'] / max(v['launches'], 1):.4f} ms"
                                                          for k, v in per.items()))
EOF
