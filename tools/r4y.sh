set -o pipefail
O=gpurun_out/r4y; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_extract_gpu.py tests/test_batched_gpu.py tests/test_match_gpu.py tests/test_capi_cpp.py tests/test_golden.py tests/test_undistort_gpu.py tests/test_sharded_gpu.py -x -q --timeout 300 --timeout-method thread > $O/front_tests.log 2>&1 || exit 1
timeout -k 10 500 python tools/lat_ab.py tools/abl/libslamgpu_nofork.so tools/abl/libslamgpu_aux.so tools/abl/libslamgpu_nofork.so tools/abl/libslamgpu_aux.so > $O/lat_ab.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/lat_trace -o run -- python3 tools/lat_loop.py > $O/lat_trace.log 2>&1
exit 0
