#!/bin/bash
# Round evidence on the current tree: the GPU parity suite, smoke(), a default bench line and a
# rocprofv3 kernel trace (stats) of the same bench command.
#   TAG=r4x tools/round_final.sh
export TMPDIR=/tmp
TAG=${TAG:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1
rc=$?
tail -3 $OUT/gpu_tests.log
grep -E "FAILED|ERROR" $OUT/gpu_tests.log | head -20
[ $rc -gt 1 ] && { echo "stop: pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 1; }
tail -c 400 $OUT/bench.json
if [ "${STATS:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
    python3 bench.py > $OUT/stats_bench.json 2> $OUT/stats.log || { echo "rocprof rc=$?"; exit 1; }
  echo "rocprof ok"
fi
echo "round_final done"
