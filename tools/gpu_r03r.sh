#!/bin/bash
# round-3 session r: on one box, the default bench line and a rocprofv3 kernel-stats run of the same
# bench (event vs rocprof agreement at the final build), then the new vs the old defaults interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { echo bench_fail; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o run -- python3 bench.py --no-cpu-baseline --no-extras > $O/prof.log 2>&1 || { echo prof_fail; exit 1; }
find $O/prof -name "*kernel_trace*" -delete
python3 - <<'PY'
import json, csv, glob
d = json.loads(open("gpurun_out/r03r/bench_c3.json").read().strip().splitlines()[-1])
print("bench", round(d["value"], 1), d["roofline"]["per_kernel"])
p = json.loads(open("gpurun_out/r03r/prof.log").read().strip().splitlines()[-1])
print("bench under rocprof", round(p["value"], 1), p["roofline"]["per_kernel"])
for r in csv.DictReader(open(glob.glob("gpurun_out/r03r/prof/**/*kernel_stats.csv", recursive=True)[0])):
    if "pass_" in r["Name"]:
        print(r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e6)
PY
for round in 1 2 3; do
  timeout -k 10 200 python3 tools/sweep.py --config c3 --steps 4 ADMM_PASSB_PMODE=2,3 ADMM_PL=0,1 >> $O/ab.txt 2>&1 || exit 1
done
grep knobs $O/ab.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['knobs'], round(d['it_s'], 1), round(d['A_ms'], 4), round(d['B_ms'], 4), d['diff_vs_first'])"
