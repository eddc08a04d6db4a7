#!/bin/bash
# One parametrised gpurun recipe (replaces the per-experiment r*.sh files):
#   tools/gpu.sh TAG step [step ...]        -> gpurun_out/TAG/...
# Steps (each under its own time limit; the first failing step ends the call):
#   tests[=PATHS]   pytest -m gpu (default: the whole suite)
#   smoke           __graft_entry__.smoke()
#   bench           python3 bench.py (default line) -> bench.json
#   quick           python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-optimizer
#   stats           rocprofv3 --kernel-trace --stats of the default bench + the timed-region split
#   traffic         FETCH_SIZE / WRITE_SIZE passes (tools/pmc_traffic.sh)
#   pipes           two --pmc passes of pipe counters (tools/pmc_pipes.sh -> tools/pipes.py)
#   pmc=GROUPFILE   one --pmc pass with the counters listed in GROUPFILE (tools/pmc_groups/)
#   ab=LIB,LIB,...  tools/ab.py A/B of library builds (bench --steps 10), run twice
#   py=SCRIPT[:ARGS] python3 SCRIPT ARGS (ARGS ':'-separated)
#   pmclibs=LIB,... one --pmc pass per library build (counters: $PMC_COUNTERS), tools/pmc_libs.sh
#   rates           tools/valu_rates (VALU issue-rate probe; build it first)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
QUICK="--steps 10 --warmup 2 --no-cpu-baseline --no-optimizer"
for s in "$@"; do
  case $s in
    tests|tests=*)
      paths=${s#tests}; paths=${paths#=}; paths=${paths//,/ }
      timeout -k 10 500 python3 -u -m pytest ${paths:-tests} -m gpu -v --timeout 200 \
        --timeout-method thread > $O/gpu_tests.log 2>&1
      rc=$?; tail -3 $O/gpu_tests.log; grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
      # test failures (rc 1) are reported and the call goes on; a crash, abort or timeout stops it
      [ $rc -gt 1 ] && { echo "stop: pytest rc=$rc"; exit $rc; } ;;
    smoke)
      timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
        || { echo "smoke rc=$?"; tail -5 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err \
        || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
      tail -c 300 $O/bench.json ;;
    quick)
      timeout -k 10 200 python3 bench.py $QUICK > $O/quick.json 2> $O/quick.err \
        || { echo "quick rc=$?"; tail -5 $O/quick.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open('$O/quick.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d.get('kernel_ms_per_step'))" ;;
    stats)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
        python3 bench.py > $O/stats_bench.json 2> $O/stats.log || { echo "rocprof rc=$?"; exit 1; }
      f=$(ls $O/stats/*/run_kernel_trace.csv $O/stats/run_kernel_trace.csv 2>/dev/null | head -1)
      [ -n "$f" ] && python3 tools/stats_timed.py $f > $O/timed_kernel_stats.csv
      echo "stats ok" ;;
    pipes)
      OUT=$O/pipes timeout -k 10 560 bash tools/pmc_pipes.sh > $O/pipes.log 2>&1 || { echo "pipes rc=$?"; cat $O/pipes.log; exit 1; }
      echo "pipes ok" ;;
    traffic)
      OUT=$O/traffic timeout -k 10 700 bash tools/pmc_traffic.sh > $O/traffic.log 2>&1 || { echo "traffic rc=$?"; exit 1; }
      echo "traffic ok" ;;
    pmc=*)
      grp=${s#pmc=}; name=$(basename $grp .txt)
      timeout -s KILL 200 rocprofv3 --pmc $(cat $grp) --kernel-trace --output-format csv \
        -d $O/pmc_$name -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline \
        --no-optimizer > $O/pmc_$name.log 2>&1 || { echo "pmc $name rc=$?"; exit 1; }
      echo "pmc $name ok" ;;
    ab=*)
      libs=${s#ab=}; libs=${libs//,/ }
      timeout -k 10 900 python3 tools/ab.py $libs $libs > $O/ab.log 2>&1 || { echo "ab rc=$?"; cat $O/ab.log; exit 1; }
      cat $O/ab.log ;;
    py=*)
      spec=${s#py=}; script=${spec%%:*}; args=""; [ "$spec" != "$script" ] && args=${spec#*:}
      timeout -k 10 600 python3 -u $script ${args//:/ } > $O/$(basename $script .py).log 2>&1 \
        || { echo "py $script rc=$?"; tail -20 $O/$(basename $script .py).log; exit 1; }
      tail -20 $O/$(basename $script .py).log ;;
    pmclibs=*)
      spec=${s#pmclibs=}; libs=${spec//,/ }
      bash tools/pmc_libs.sh $O/pmclibs "${PMC_COUNTERS:-SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU}" $libs \
        > $O/pmclibs.log 2>&1 || { echo "pmclibs rc=$?"; tail $O/pmclibs.log; exit 1; }
      cat $O/pmclibs.log ;;
    rates)
      timeout -k 10 120 ./tools/valu_rates > $O/valu_rates.txt 2>&1 || { echo "rates rc=$?"; exit 1; }
      cat $O/valu_rates.txt ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "gpu.sh $TAG done"
