set -o pipefail
for flags in "--no-cpu-baseline --no-optimizer --no-bow" "--no-optimizer --no-bow" "--no-cpu-baseline --no-bow" "--no-cpu-baseline --no-optimizer"; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 $flags > gpurun_out/h2d_ab.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/h2d_ab.json').read().strip().splitlines()[-1]); h=d['drop_in']['batched_h2d']; print(sys.argv[1:], h['value'], h['ms_per_step'], h['copy_ms_per_step'], h['compute_ms_per_step'])" $flags
done
