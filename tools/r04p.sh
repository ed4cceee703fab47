#!/bin/bash
# Round 4, call p: the extended early-stop hand-off test (256 x 256 at batch 1 / 2: 8 norm copies).
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "handoff" \
  > gpurun_out/r04p_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r04p_gpu_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r04p_gpu_tests.log | tail -12
