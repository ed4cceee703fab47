#!/bin/bash
# Round 4, call r: the new W % 4 != 0 / H*W % 4 == 0 cases of the fused DNN passes.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_dnn.py -m gpu -x -v --timeout 300 --timeout-method thread -k "odd_plane or ula_chains" \
  > gpurun_out/r04r_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r04r_gpu_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r04r_gpu_tests.log | tail -12
