set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_generic.py tests/test_gpu_0_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/generic_tests.log 2>&1 || { echo tests_fail; tail -30 gpurun_out/generic_tests.log; exit 1; }
tail -3 gpurun_out/generic_tests.log
TAG=r02y_bsd BENCH_ARGS="--config bsd" bash tools/gpu_bench_prof.sh
