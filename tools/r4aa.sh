set -o pipefail
O=gpurun_out/r4aa; mkdir -p $O
SLAMGPU_PYR_BANDS=1 timeout -k 10 400 python -u -m pytest tests/test_extract_gpu.py tests/test_batched_gpu.py tests/test_match_gpu.py tests/test_capi_cpp.py tests/test_golden.py tests/test_sharded_gpu.py -x -q --timeout 300 --timeout-method thread > $O/front_tests.log 2>&1 || exit 1
timeout -k 10 700 python tools/ab_env.py - SLAMGPU_PYR_BANDS=1 - SLAMGPU_PYR_BANDS=1 > $O/bench_ab.log 2>&1 || exit 1
exit 0
