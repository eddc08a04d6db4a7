set -o pipefail
O=gpurun_out/r4aj; mkdir -p $O
A=tools/abl/libslamgpu_
timeout -k 10 300 python -u -m pytest tests/test_eg_gpu.py tests/test_sim3_gpu.py -x -q --timeout 120 --timeout-method thread > $O/eg_tests.log 2>&1 || exit 1
timeout -k 10 600 python tools/eg_ab.py ${A}head.so ${A}eglin.so ${A}head.so ${A}eglin.so > $O/eg_ab.log 2>&1 || exit 1
exit 0
