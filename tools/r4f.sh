set -o pipefail
O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 500 python tools/ab.py tools/abl/libslamgpu_base.so tools/abl/libslamgpu_od4.so tools/abl/libslamgpu_od5.so tools/abl/libslamgpu_base.so tools/abl/libslamgpu_od4.so tools/abl/libslamgpu_od5.so > $O/ab.log 2>&1 &&
for v in od4 od5; do SLAMGPU_LIB=$(realpath tools/abl/libslamgpu_$v.so) timeout -k 10 300 python -u -m pytest tests/test_extract_gpu.py tests/test_batched_gpu.py tests/test_golden.py -x -q --timeout 200 --timeout-method thread > $O/parity_$v.log 2>&1 || exit 1; done &&
timeout -k 10 400 python tools/pose_lat_ab.py tools/abl/libslamgpu_pm0.so tools/abl/libslamgpu_pm1.so tools/abl/libslamgpu_pm0.so tools/abl/libslamgpu_pm1.so > $O/pose_ab.log 2>&1 &&
SLAMGPU_LIB=$(realpath tools/abl/libslamgpu_pm1.so) timeout -k 10 400 python -u -m pytest tests/test_pose_gpu.py tests/test_capi_cpp.py -x -q --timeout 300 --timeout-method thread > $O/pose_tests_pm1.log 2>&1
