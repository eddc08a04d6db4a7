set -o pipefail
O=gpurun_out/r4u; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_eg_gpu.py -x -q --timeout 300 --timeout-method thread > $O/eg_tests.log 2>&1 || exit 1
timeout -k 10 400 python tools/eg_ab.py tools/abl/libslamgpu_head.so tools/abl/libslamgpu_egbk.so tools/abl/libslamgpu_egbk2.so tools/abl/libslamgpu_head.so tools/abl/libslamgpu_egbk.so tools/abl/libslamgpu_egbk2.so > $O/eg_ab.log 2>&1 || exit 1
exit 0
