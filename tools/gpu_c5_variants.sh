#!/bin/bash
# C5 training step under framework options: MIOpen find (cudnn.benchmark), NHWC activations
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for opt in "" "--c5-conv-benchmark" "--c5-channels-last" "--c5-channels-last --c5-conv-benchmark"; do
  tag=$(echo "x$opt" | tr -d ' -')
  timeout -k 10 500 python -u bench.py --config c5 --steps 3 --warmup 1 $opt > gpurun_out/c5v_$tag.json 2> gpurun_out/c5v_$tag.err || { echo "fail $opt"; exit 1; }
done
echo done
