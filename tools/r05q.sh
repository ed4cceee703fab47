#!/bin/bash
# round 5 call q: tile kernel: untracked and tracked inner iterations as separate loops (compile-time rel-err tracking) (prod)
# vs the committed kernel (head)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "tile or redo or early_stop or handoff" > gpurun_out/r05q_parity.log 2>&1 || { tail -40 gpurun_out/r05q_parity.log; exit 1; }
tail -1 gpurun_out/r05q_parity.log
tools/ab_bench.sh r05q8 3 "--steps 400 --warmup 40 --batch 8" prod head || exit 1
tools/ab_bench.sh r05qc 3 "--steps 400 --warmup 40 --batch 1 --H 481 --W 321" prod head || exit 1
tools/ab_bench.sh r05q16 2 "--steps 400 --warmup 40 --batch 16" prod head || exit 1
