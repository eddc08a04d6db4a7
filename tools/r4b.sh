set -o pipefail
O=gpurun_out/r4b; mkdir -p $O
timeout -k 10 120 tools/valu_rates > $O/valu_rates.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_extract_gpu.py tests/test_batched_gpu.py tests/test_edge_gpu.py tests/test_golden.py tests/test_capi_cpp.py tests/test_match_gpu.py -x -v --timeout 200 --timeout-method thread > $O/parity.log 2>&1 &&
timeout -k 10 400 python tools/ab.py tools/abl/libslamgpu_base.so tools/abl/libslamgpu_od1.so tools/abl/libslamgpu_base.so tools/abl/libslamgpu_od1.so > $O/ab.log 2>&1 &&
GROUPS_FILE=tools/pmc_groups/issue.txt KERNEL="orient_desc" OUT=$O/pmc \
  tools/pmc_run.sh python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-optimizer --no-bow --no-latency &&
python3 tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt
