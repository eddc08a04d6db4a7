set -o pipefail
O=gpurun_out/r4ah; mkdir -p $O
A=tools/abl/libslamgpu_
timeout -k 10 500 python tools/pose_lat_ab.py ${A}pswap.so ${A}pw4.so ${A}pswap.so ${A}pw4.so > $O/pose_ab.log 2>&1 || exit 1
exit 0
