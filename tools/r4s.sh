set -o pipefail
O=gpurun_out/r4s; mkdir -p $O
SLAMGPU_OCT_LVL=1 timeout -k 10 400 python -u -m pytest tests/test_batched_gpu.py tests/test_extract_gpu.py -x -q --timeout 300 --timeout-method thread > $O/batched_lvl_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest tests/test_batched_gpu.py tests/test_extract_gpu.py tests/test_golden.py -x -q --timeout 300 --timeout-method thread > $O/front_tests.log 2>&1 || exit 1
timeout -k 10 700 python tools/ab_env.py - SLAMGPU_OCT_LVL=1 - SLAMGPU_OCT_LVL=1 > $O/ab.log 2>&1 || exit 1
exit 0
