set -o pipefail
O=gpurun_out/r4a; mkdir -p $O
timeout -k 10 120 tools/valu_rates > $O/valu_rates.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_sharded_gpu.py -x -v --timeout 200 --timeout-method thread > $O/sharded.log 2>&1 &&
GROUPS_FILE=tools/pmc_groups/issue.txt KERNEL="orient_desc|fast_cells|pyr_down|octree_img|stereo_match|search_resolve|search_cand" OUT=$O/pmc \
  tools/pmc_run.sh python3 bench.py --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-optimizer --no-bow --no-latency &&
python3 tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt
