#!/bin/bash
# Round-3 GPU call: the GPU parity suite, a default bench line, then the cooperative-launch
# experiment (C5 LocalBA under rocprofv3 with the plain launch, then with the runtime's
# cooperative launch -- the variant that crashed at exit in round 2 runs last).
#   TAG=r3a tools/r3_tests_bench.sh
export TMPDIR=/tmp
TAG=${TAG:-r3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  ${TESTS:-} > $OUT/gpu_tests.log 2>&1
rc=$?
tail -4 $OUT/gpu_tests.log
[ $rc -gt 1 ] && { echo "stop: pytest rc=$rc"; exit $rc; }
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python3 bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; exit 3; }
  tail -c 600 $OUT/bench.json
fi
if [ -n "${AB:-}" ]; then  # A/B of library builds: AB="tools/abl/libslamgpu_x.so slam_framework_amd/libslamgpu.so"
  timeout -k 10 600 python3 tools/ab.py $AB $AB > $OUT/ab.log 2>&1
  echo "ab rc=$?"; cat $OUT/ab.log
fi
if [ -n "${PMC_LIBS:-}" ]; then  # one PMC pass per library over a short single-batch bench
  i=0
  for lib in $PMC_LIBS; do
    i=$((i+1))
    SLAMGPU_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES} \
      --kernel-include-regex "${PMC_RE:-orient_desc}" --kernel-trace --output-format csv \
      -d $OUT/pmc$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline \
      --no-optimizer --no-bow --no-latency --inflight 1 > $OUT/pmc$i.log 2>&1
    echo "pmc $lib rc=$?"
  done
fi
if [ "${LAT:-0}" = "1" ]; then  # the single-frame drop-in call: per-kernel trace
  timeout -k 10 120 python3 tools/latency_probe.py > $OUT/lat.log 2>&1
  echo "latency probe rc=$?"; cat $OUT/lat.log
  SLAMGPU_FRAME_GRAPH=0 timeout -k 10 120 python3 tools/latency_probe.py > $OUT/lat_eager.log 2>&1
  echo "latency probe (eager launches) rc=$?"; grep frame_stereo $OUT/lat_eager.log
  timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/lat -o run -- \
    python3 tools/latency_probe.py > $OUT/lat_prof.log 2>&1
  echo "latency trace rc=$?"
  if [ -f tools/abl/libslamgpu_octprof.so ]; then  # octree phase wall clocks (printf build)
    SLAMGPU_LIB=$PWD/tools/abl/libslamgpu_octprof.so timeout -k 10 120 python3 tools/latency_probe.py \
      > $OUT/lat_octprof.log 2>&1
    echo "octree phase probe rc=$?"
  fi
fi
if [ "${COOP:-0}" = "1" ]; then
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/plain -o run -- \
    python3 tools/ba_latency.py 3 --ba-only > $OUT/plain.log 2>&1
  echo "plain launch under rocprofv3: rc=$?"
  SLAMGPU_BA_COOP_LAUNCH=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/coop -o run -- python3 tools/ba_latency.py 3 --ba-only > $OUT/coop.log 2>&1
  echo "cooperative launch under rocprofv3: rc=$?"
fi
echo "r3 call done"
