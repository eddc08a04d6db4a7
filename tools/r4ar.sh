set -o pipefail
O=gpurun_out/r4ar; mkdir -p $O
A=tools/abl/libslamgpu_
timeout -k 10 400 python -u -m pytest tests/test_pose_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pose_tests.log 2>&1 || exit 1
timeout -k 10 500 python tools/pose_lat_ab.py ${A}pcur.so ${A}pnobr.so ${A}pcur.so ${A}pnobr.so > $O/pose_ab.log 2>&1 || exit 1
exit 0
