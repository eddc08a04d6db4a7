#!/bin/bash
# Round-3 fused-pyramid call: the GPU parity suite, then an A/B of the pyramid variants
# (SLAMGPU_PYR_FUSED=0: one pyr_down launch per level; SLAMGPU_PYR_NB: bands per image).
#   TAG=r3t VARIANTS="- SLAMGPU_PYR_FUSED=0" tools/r3_pyr.sh
export TMPDIR=/tmp
TAG=${TAG:-r3t}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  ${TESTS:-} > $OUT/gpu_tests.log 2>&1
rc=$?
tail -4 $OUT/gpu_tests.log
grep -E "FAILED|ERROR" $OUT/gpu_tests.log | head -20
[ $rc -gt 1 ] && { echo "stop: pytest rc=$rc"; exit $rc; }
if [ -n "${VARIANTS:-}" ]; then
  timeout -k 10 900 python3 tools/ab_env.py $VARIANTS -- ${AB_ARGS:---steps 10 --warmup 2 --no-cpu-baseline --no-optimizer --no-bow} > $OUT/ab.log 2>&1
  echo "ab rc=$?"; cat $OUT/ab.log
fi
echo "r3_pyr done"
