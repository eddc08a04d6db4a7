set -e
export TMPDIR=/tmp
O=gpurun_out/r2v
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/solo -o run -- python3 bench.py --inflight 1 --no-optimizer --no-bow --no-latency --no-cpu-baseline --steps 10 > $O/solo.log 2>&1
OUT=$O/pmc timeout -k 10 500 tools/pmc_stalls.sh > $O/pmc.log 2>&1
echo done
