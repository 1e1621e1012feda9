set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/m3
MIXED_SWEEP3=1 timeout -k 10 200 tools/membench/stream_mimic > gpurun_out/m3/time.txt 2>&1 || exit 1
MIXED_SWEEP3=1 ONCE=1 timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d gpurun_out/m3/rd -o run -- tools/membench/stream_mimic > gpurun_out/m3/rd.log 2>&1 || exit 1
MIXED_SWEEP3=1 ONCE=1 timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d gpurun_out/m3/wr -o run -- tools/membench/stream_mimic > gpurun_out/m3/wr.log 2>&1 || exit 1
echo m3_ok
