#!/bin/bash
# Round-4 verification + A/B session (through gpurun): the mixed-path tests, HD pass-B plane groups
# (ADMM_PASSB_M_GP 1 vs the model), the HD bench line, and the BSD row-inverse occupancy variant
# (tools/_variants/inv4.so) interleaved with the default library.  Each GPU step has its own time limit;
# a crash, abort or timeout ends the session.  -> gpurun_out/r04e/, gpurun_out/ab_*.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash tools/gpu_session.sh r04e "mixed or gfused" nobench || exit $?
: > gpurun_out/ab_hd_gp.txt
for g in 1 0 1 0; do
  ADMM_PASSB_M_GP=$g timeout -k 10 120 python tools/sweep.py --config hd --steps 5 >> gpurun_out/ab_hd_gp.txt 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --config hd --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_hd.json 2> gpurun_out/bench_hd.err || exit 1
: > gpurun_out/ab_inv4.txt
for v in "" tools/_variants/inv4.so "" tools/_variants/inv4.so; do
  echo "lib=${v:-default}" >> gpurun_out/ab_inv4.txt
  ADMMTOR_LIB_OVERRIDE=$v timeout -k 10 200 python bench.py --config bsd --steps 10 --warmup 2 --no-cpu-baseline \
    --no-parity >> gpurun_out/ab_inv4.txt 2>/dev/null || exit 1
done
echo round_session_done
