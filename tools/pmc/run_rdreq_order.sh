set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
RD="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
for o in 0 1; do
  ADMM_PASSB_ORDER=$o timeout -s KILL 180 rocprofv3 --pmc $RD --output-format csv -d gpurun_out/rdo/o$o -o run -- python3 tools/sweep.py --config c3 --steps 1 --maxit 10 > gpurun_out/rdo/o$o.log 2>&1 || exit 1
done
echo ok
