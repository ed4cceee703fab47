#!/bin/bash
# 32-row tiles in the auto dispatch: tile / dispatch / CLI tests, then castle and 8-chain timing.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_cli.py -k "tile or auto_dispatch or single_channel or cli" > gpurun_out/r03q_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r03q_tests.log
[ $rc -ne 0 ] && { grep -m3 -A40 "^____" gpurun_out/r03q_tests.log | head -80; exit 1; }
for args in "--batch 1 --H 481 --W 321" "--batch 1 --H 321 --W 481" "--batch 1" "--batch 3" "--batch 8"; do
  r=$(timeout -k 10 120 python3 bench.py --no-cpu --steps 200 --warmup 20 --warmup-seconds 0.3 $args 2>/dev/null | tail -1) || exit 1
  echo "$args $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel"], d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
timeout -k 10 300 python3 tools/castle_timing.py 10000 1
