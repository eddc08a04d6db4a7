for inf in 1 2 3 1 2; do
  timeout -k 10 200 python3 bench.py --inflight $inf --steps 30 --no-cpu-baseline --no-optimizer --no-bow --no-latency 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('inflight', $inf, d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
