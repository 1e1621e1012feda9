#!/bin/bash
# Plane parts (HIP streams) of the BSD solve on the odd-length path: bench.py --config bsd at
# ADMM_GEN_STREAMS = 1 .. 4 (a release runtime setting), two interleaved rounds -> gpurun_out/streams_bsd.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/streams_bsd.txt
: > "$OUT"
for round in 1 2; do
  for n in 1 2 3 4; do
    echo "round $round streams $n" >> "$OUT"
    ADMM_GEN_STREAMS=$n timeout -k 10 200 python3 bench.py --config bsd --steps 10 --warmup 2 --no-cpu-baseline \
      --no-parity 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])" >> "$OUT" || exit 1
  done
done
cat "$OUT"
