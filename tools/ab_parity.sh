#!/bin/bash
# Extraction/matching parity of each A/B build: tools/ab_parity.sh lib1.so lib2.so ...
set -e
for lib in "$@"; do
  SLAMGPU_LIB=$(realpath $lib) timeout -k 10 300 python -u -m pytest tests/test_extract_gpu.py tests/test_batched_gpu.py tests/test_edge_gpu.py tests/test_match_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parity_$(basename $lib).log 2>&1
  echo "$lib parity ok"
done
