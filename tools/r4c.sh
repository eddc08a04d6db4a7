set -o pipefail
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 400 python tools/ab.py tools/abl/libslamgpu_base.so tools/abl/libslamgpu_od1.so tools/abl/libslamgpu_base.so tools/abl/libslamgpu_od1.so > $O/ab.log 2>&1 &&
timeout -k 10 500 python tools/eg_ab.py tools/abl/libslamgpu_od1.so tools/abl/libslamgpu_egl.so tools/abl/libslamgpu_od1.so tools/abl/libslamgpu_egl.so > $O/eg_ab.log 2>&1 &&
SLAMGPU_LIB=$(realpath tools/abl/libslamgpu_egl.so) timeout -k 10 300 python -u -m pytest tests/test_eg_gpu.py -x -v --timeout 200 --timeout-method thread > $O/eg_tests_egl.log 2>&1 &&
GROUPS_FILE=tools/pmc_groups/issue.txt KERNEL="orient_desc" OUT=$O/pmc \
  tools/pmc_run.sh python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-optimizer --no-bow --no-latency &&
python3 tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt
