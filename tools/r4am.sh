set -o pipefail
O=gpurun_out/r4an; mkdir -p $O
A=tools/abl/libslamgpu_
timeout -k 10 600 python tools/eg_ab.py ${A}egcur.so ${A}egz.so ${A}egcur.so ${A}egz.so > $O/eg_ab.log 2>&1 || exit 1
exit 0
