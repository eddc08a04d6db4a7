export TMPDIR=/tmp
mkdir -p gpurun_out/r2b
timeout -k 10 300 python3 -u -m pytest tests/test_batched_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r2b/batched.log 2>&1
echo "pytest rc=$?"; tail -12 gpurun_out/r2b/batched.log
SLAMGPU_BENCH_GATHER=1 timeout -k 10 300 python3 bench.py --no-optimizer --no-bow --no-cpu-baseline > gpurun_out/r2b/bench_gather.json 2> gpurun_out/r2b/bench_gather.err
echo "bench rc=$?"; tail -c 1500 gpurun_out/r2b/bench_gather.json; tail -5 gpurun_out/r2b/bench_gather.err
