set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6i; mkdir -p $O
timeout -k 10 120 python3 tools/eg_time.py 400 > $O/eg400.log 2>&1 && timeout -k 10 180 python3 tools/eg_time.py 1000 > $O/eg1000.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/eg_time.py 400 > $O/prof.log 2>&1
cat $O/eg400.log $O/eg1000.log
