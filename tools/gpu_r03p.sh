#!/bin/bash
# round-3 session p: combinations of the fused path's order / layout knobs (pass B tile order, pass A
# plane order, lane-paired layout, two-stream halves), interleaved in one process, 4 rounds, C3 and C2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
for round in 1 2 3 4; do
  timeout -k 10 300 python3 tools/sweep.py --config c3 --steps 4 ADMM_PASSB_PMODE=3,2 ADMM_PASSA_REV=0,1 ADMM_PL=1,0 >> $O/c3.txt 2>&1 || exit 1
  timeout -k 10 200 python3 tools/sweep.py --config c3 --steps 4 ADMM_PASSB_PMODE=2 ADMM_PL=0 ADMM_STREAMS=1,2 >> $O/c3s.txt 2>&1 || exit 1
done
for round in 1 2; do
  timeout -k 10 200 python3 tools/sweep.py --config c2 --steps 10 ADMM_PASSB_PMODE=3,2 ADMM_PL=1,0 >> $O/c2.txt 2>&1 || exit 1
  timeout -k 10 200 python3 tools/sweep.py --config c3iso --steps 4 ADMM_PASSB_PMODE=3,2 ADMM_PL=1,0 >> $O/c3iso.txt 2>&1 || exit 1
done
for f in c3 c3s c2 c3iso; do
  echo "== $f"
  grep knobs $O/$f.txt | python3 -c "
import sys, json, collections
acc = collections.defaultdict(list)
for l in sys.stdin:
    d = json.loads(l); acc[json.dumps(d['knobs'])].append((d['it_s'], d['A_ms'], d['B_ms'], d['diff_vs_first']))
for k, v in acc.items():
    print(k, 'it/s', [round(x[0], 1) for x in v], 'A', round(sum(x[1] for x in v) / len(v), 4), 'B', round(sum(x[2] for x in v) / len(v), 4), 'diff', max(x[3] for x in v))"
done
