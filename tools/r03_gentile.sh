#!/bin/bash
# Tile kernel with padded rows / column segments: parity tests, then B = 1 / 2 real-shape timing.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "tile or auto_dispatch or padded or segmented" > gpurun_out/r03k_gentile_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r03k_gentile_tests.log
[ $rc -ne 0 ] && { grep -m3 -A40 "^____" gpurun_out/r03k_gentile_tests.log | head -80; exit 1; }
for args in "--batch 1 --H 481 --W 321" "--batch 1 --H 321 --W 481" "--batch 2 --H 481 --W 321" "--batch 2 --H 321 --W 481" "--batch 8" "--batch 4 --H 481 --W 321"; do
  r=$(timeout -k 10 120 python3 bench.py --no-cpu --steps 200 --warmup 20 --warmup-seconds 0.5 $args | tail -1) || exit 1
  echo "$args => $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel"], d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
