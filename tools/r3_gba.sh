#!/bin/bash
# Round-3 grid-factorisation call: the BA / GBA parity tests, then the map-scale GBA timing with
# the grid factorisation (default) and with work-group 0 alone (SLAMGPU_GBA_MWG=0).
#   TAG=r3x tools/r3_gba.sh
export TMPDIR=/tmp
TAG=${TAG:-r3x}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest ${TESTS:-tests/test_gba_gpu.py tests/test_ba_gpu.py} -m gpu -v \
  --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
tail -4 $OUT/gpu_tests.log
grep -E "FAILED|ERROR|Error" $OUT/gpu_tests.log | head -20
[ $rc -gt 1 ] && { echo "stop: pytest rc=$rc"; exit $rc; }
SLAMGPU_BA_PROFILE=1 timeout -k 10 120 python3 tools/gba_profile.py 1500 > $OUT/gba_grid.log 2>&1 || { echo "gba grid rc=$?"; cat $OUT/gba_grid.log | tail; exit 1; }
cat $OUT/gba_grid.log
SLAMGPU_GBA_MWG=0 SLAMGPU_BA_PROFILE=1 timeout -k 10 120 python3 tools/gba_profile.py 1500 > $OUT/gba_wg0.log 2>&1 || { echo "gba wg0 rc=$?"; exit 1; }
cat $OUT/gba_wg0.log
echo "r3_gba done"
