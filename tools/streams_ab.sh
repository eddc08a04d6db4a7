#!/bin/bash
# bench.py quick runs with 1 or 2 contexts (streams) per batch, alternating, twice each
set -o pipefail
for rep in 1 2; do
  for ns in 1 2; do
    timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-optimizer --no-bow --no-latency --no-alone --streams $ns > gpurun_out/streams_ab.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/streams_ab.json').read().strip().splitlines()[-1]); print('streams', sys.argv[1], d['ms_per_step'], d['value'])" $ns
  done
done
