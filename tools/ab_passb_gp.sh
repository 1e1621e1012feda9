#!/bin/bash
# pass B plane groups per block (ADMM_PASSB_GP) x library variants (tools/_variants/*.so + the
# in-tree build), C3, interleaved rounds.  Each GPU step has its own time limit.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for round in 1 2; do
  for v in torch-admm-deconv_amd/admmtor/_lib/libadmm_tv.so tools/_variants/*.so; do
    echo "== $v round $round"
    ADMMTOR_LIB_OVERRIDE=$v timeout -k 10 200 python3 tools/sweep.py --config ${CFG:-c3} --steps 3 ADMM_PASSB_GP=${GPS:-1,2,4,8} || exit 1
  done
done
