set -o pipefail
O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 500 python tools/ab.py tools/abl/libslamgpu_base.so tools/abl/libslamgpu_odA.so tools/abl/libslamgpu_odB.so tools/abl/libslamgpu_base.so tools/abl/libslamgpu_odA.so tools/abl/libslamgpu_odB.so > $O/ab.log 2>&1 &&
for v in odA odB; do SLAMGPU_LIB=$(realpath tools/abl/libslamgpu_$v.so) timeout -k 10 300 python -u -m pytest tests/test_extract_gpu.py tests/test_batched_gpu.py tests/test_golden.py -x -q --timeout 200 --timeout-method thread > $O/parity_$v.log 2>&1 || exit 1; done
