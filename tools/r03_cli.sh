#!/bin/bash
# CLI batching / sharding tests, the castle known answer, castle timing (B = 1 and 64).
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_cli.py > $out/r03f_cli_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $out/r03f_cli_tests.log | tail -15
[ $rc -ne 0 ] && { grep -m3 -A30 "^____" $out/r03f_cli_tests.log | head -80; exit 1; }
timeout -k 10 300 python tools/castle_timing.py 10000 1 > $out/r03f_castle_b1.json && cat $out/r03f_castle_b1.json
timeout -k 10 300 python tools/castle_timing.py 2000 64 > $out/r03f_castle_b64.json && cat $out/r03f_castle_b64.json
