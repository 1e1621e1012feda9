#!/bin/bash
# round-3 session i: the column-walking fused step (ADMM_GSTEP_CW) -- generic GPU tests on the new
# library, then interleaved A/B of the old (cw0) and new (cw1) item: bench.py --config bsd and the
# generic size sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03i
timeout -k 10 600 python -u -m pytest tests/test_gpu_generic.py tests/test_gpu_gcol_mm.py tests/test_gpu_concurrency.py \
    -q -m gpu -rfE --timeout 300 --timeout-method thread > gpurun_out/r03i/tests.log 2>&1
rc=$?
echo "tests_exit=$rc"
tail -5 gpurun_out/r03i/tests.log
[ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do
  for v in cw0 cw1; do
    echo "== $v round $round" >> gpurun_out/r03i/ab.txt
    ADMMTOR_LIB_OVERRIDE=tools/_variants/$v.so timeout -k 10 200 python3 bench.py --config bsd --steps 5 \
        --no-cpu-baseline --no-parity >> gpurun_out/r03i/ab.txt 2>&1 || exit 1
  done
done
python3 - <<'PY'
import json
cur = None
for line in open("gpurun_out/r03i/ab.txt"):
    if line.startswith("=="):
        cur = line.strip()
    elif line.startswith("{"):
        d = json.loads(line)
        pk = d["roofline"]["per_kernel"]
        print(cur, round(d["value"]), {k: round(v["ms_total"] / max(v["launches"], 1), 4) for k, v in pk.items()})
PY
for v in cw0 cw1; do
  echo "== sizes $v" >> gpurun_out/r03i/sizes.txt
  ADMMTOR_LIB_OVERRIDE=tools/_variants/$v.so timeout -k 10 300 python3 tools/bench_generic_sizes.py >> gpurun_out/r03i/sizes.txt 2>&1 || exit 1
done
cat gpurun_out/r03i/sizes.txt
