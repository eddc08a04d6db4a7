set -o pipefail
O=gpurun_out/r4w; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_extract_gpu.py tests/test_batched_gpu.py tests/test_match_gpu.py tests/test_capi_cpp.py tests/test_golden.py -x -q --timeout 300 --timeout-method thread > $O/front_tests.log 2>&1 || exit 1
timeout -k 10 500 python tools/lat_ab.py tools/abl/libslamgpu_b0.so tools/abl/libslamgpu_band.so tools/abl/libslamgpu_band.so:SLAMGPU_FORK=0 tools/abl/libslamgpu_b0.so tools/abl/libslamgpu_band.so tools/abl/libslamgpu_band.so:SLAMGPU_FORK=0 > $O/lat_ab.log 2>&1 || exit 1
timeout -k 10 700 python tools/ab.py tools/abl/libslamgpu_band.so tools/abl/libslamgpu_oimg.so tools/abl/libslamgpu_band.so tools/abl/libslamgpu_oimg.so > $O/bench_ab.log 2>&1 || exit 1
exit 0
