#!/bin/bash
# gpurun with retries ONLY for gpurun's own "no box / infrastructure" answer (exit code 3: nothing
# ran on a GPU, nothing charged). Any other exit code -- including a failing or timed-out GPU
# command -- is returned at once, never retried.
#   tools/gpurun_retry.sh <gpurun --timeout> '<command>' > log
T=$1; shift
for attempt in $(seq 1 ${ATTEMPTS:-8}); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpurun_retry] attempt $attempt: no box (rc 3); waiting 90 s"
  sleep 90
done
exit 3
