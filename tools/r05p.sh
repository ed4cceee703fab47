#!/bin/bash
# round 5 call p: tile kernel: the rows' in-image / core flags as bits of two wave-uniform ints instead of bool arrays (prod)
# vs the committed kernel (head)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "tile or redo or early_stop or handoff" > gpurun_out/r05p_parity.log 2>&1 || { tail -40 gpurun_out/r05p_parity.log; exit 1; }
tail -1 gpurun_out/r05p_parity.log
tools/ab_bench.sh r05p8 3 "--steps 400 --warmup 40 --batch 8" prod head || exit 1
tools/ab_bench.sh r05pc 3 "--steps 400 --warmup 40 --batch 1 --H 481 --W 321" prod head || exit 1
tools/ab_bench.sh r05p16 2 "--steps 400 --warmup 40 --batch 16" prod head || exit 1
