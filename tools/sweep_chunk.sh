# chunked aniso forward sweep (ADMM_CHUNK planes per chunk, ADMM_STREAMS side streams)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() { echo "$1" >> gpurun_out/chunk_sweep.txt; env $1 timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity >> gpurun_out/chunk_sweep.txt 2>>gpurun_out/chunk_sweep.err; }
run "ADMM_CHUNK=0" || exit 1
for c in 3 4 6 8 12; do for n in 2 3 4; do run "ADMM_CHUNK=$c ADMM_STREAMS=$n" || exit 1; done; done
