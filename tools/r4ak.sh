set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ak; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o eg -- python3 tools/eg_trace.py 100 > $O/eg_trace.log 2>&1 || exit 1
exit 0
