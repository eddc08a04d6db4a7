#!/bin/bash
# One gpurun call: the GPU parity suite, smoke(), then the round evidence (tools/round_profile.sh).
# Test failures (pytest rc 1) do not stop the call; a timeout, abort or crash (rc > 1) does.
#   TAG=r1h tools/gpu_round.sh
export TMPDIR=/tmp
TAG=${TAG:-run}
mkdir -p gpurun_out/$TAG
run() {
  "$@"
  local rc=$?
  if [ $rc -gt 1 ]; then
    echo "stop: rc=$rc from: $*"
    exit $rc
  fi
  return 0
}
run timeout -k 10 400 python3 -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  > gpurun_out/$TAG/gpu_tests.log 2>&1
tail -3 gpurun_out/$TAG/gpu_tests.log
run timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" \
  > gpurun_out/$TAG/smoke.log 2>&1
tail -1 gpurun_out/$TAG/smoke.log
[ "${PROFILE:-1}" = "1" ] && TAG=$TAG tools/round_profile.sh
echo "gpu_round done"
