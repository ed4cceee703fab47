#!/bin/bash
# GPU test run with a per-test time limit; log under gpurun_out/.  Usage: tools/gpu_tests.sh [pytest -k expr]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/gpu_tests.log 2>&1
else
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
fi
rc=$?
tail -30 gpurun_out/gpu_tests.log
exit $rc
