#!/bin/bash
# Round 4, call n: the row stream's segment-edge cases as per-lane selects (product) against the branches between two
# inlined copies of the dual / primal (segbr); stream parity tests.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "stream or fused or padded or early_stop or multichain or config1" \
  > gpurun_out/r04n_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r04n_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04n_gpu_tests.log
tools/ab_bench.sh n64 3 "--steps 400 --warmup 40" prod segbr || exit 1
tools/ab_bench.sh n481 2 "--steps 100 --warmup 10 --warmup-seconds 0.5 --H 481 --W 321" prod segbr || exit 1
tools/ab_bench.sh n321 2 "--steps 100 --warmup 10 --warmup-seconds 0.5 --H 321 --W 481" prod segbr || exit 1
tools/ab_bench.sh n32 2 "--steps 200 --warmup 20 --warmup-seconds 0.5 --batch 32" prod segbr || exit 1
