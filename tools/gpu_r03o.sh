#!/bin/bash
# round-3 session o: re-check the fused path's runtime defaults on the final build (interleaved,
# in-process tools/sweep.py; diff_vs_first shows whether a knob changes bits): strip height, pass A
# plane order, pass B tile order / groups, two-stream halves, lane-paired layout.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
for round in 1 2; do
  timeout -k 10 200 python3 tools/sweep.py --config c3 --steps 3 ADMM_PASSA_R=8,16 ADMM_PASSA_REV=0,1 >> $O/sweep.txt 2>&1 || exit 1
  timeout -k 10 200 python3 tools/sweep.py --config c3 --steps 3 ADMM_PASSB_PMODE=3,1,2 ADMM_PASSB_GROUP=2,1 >> $O/sweep.txt 2>&1 || exit 1
  timeout -k 10 200 python3 tools/sweep.py --config c3 --steps 3 ADMM_STREAMS=1,2 ADMM_PL=1,0 >> $O/sweep.txt 2>&1 || exit 1
done
grep knobs $O/sweep.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['knobs'], round(d['it_s'], 1), round(d['A_ms'], 4), round(d['B_ms'], 4), d['diff_vs_first'])"
