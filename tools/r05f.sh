#!/bin/bash
# Round 5, call f: the multi-step tile kernel (tv_tile_ms_kernel).  Parity against one launch per step (exact and
# fast, stops never / sometimes / always), then the 8-chain step and castle at batch 1 with 0 / 10 / 20 steps
# per launch, interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "multi_step" > gpurun_out/r05f_parity.log 2>&1
rc=$?; tail -12 gpurun_out/r05f_parity.log; [ $rc -eq 0 ] || exit $rc
tools/ab_bench.sh r05f8 2 "--steps 400 --warmup 40 --batch 8" prod "prod10@--tile-multi-steps 10" "prod20@--tile-multi-steps 20" || exit 1
tools/ab_bench.sh r05fc 2 "--steps 400 --warmup 40 --batch 1 --H 481 --W 321" prod "prod10@--tile-multi-steps 10" "prod20@--tile-multi-steps 20" || exit 1
