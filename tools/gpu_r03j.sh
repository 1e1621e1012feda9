#!/bin/bash
# round-3 session j: phased plane parts (ADMM_GEN_PHASE: the parts' column passes take turns) vs the
# free-running parts, interleaved in one process (tools/sweep.py; diff_vs_first must stay 0), BSD with
# 2 and 3 parts, then the generic size sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03j
for round in 1 2 3; do
  timeout -k 10 200 python3 tools/sweep.py --config bsd --steps 5 ADMM_GEN_STREAMS=2,3 ADMM_GEN_PHASE=0,1 \
      >> gpurun_out/r03j/phase_bsd.txt 2>&1 || { tail -5 gpurun_out/r03j/phase_bsd.txt; exit 1; }
done
grep knobs gpurun_out/r03j/phase_bsd.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['knobs'], round(d['it_s']), round(d['A_ms'], 4), round(d['B_ms'], 4), d['diff_vs_first'])"
timeout -k 10 300 python3 tools/bench_generic_sizes.py ADMM_GEN_PHASE=0,1 > gpurun_out/r03j/sizes.txt 2>&1 || exit 1
cat gpurun_out/r03j/sizes.txt
