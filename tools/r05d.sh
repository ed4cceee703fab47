#!/bin/bash
# Round 5, call d: the parallel early-stop redo (ABI 11).  GPU parity suite (early-stop cases: stream / tile vs oracle,
# parallel == serial redo), the step A/B against the library before it (exp_libs/lib_base.so) at 64 and 8 chains,
# and a forced-stop run (tol 0.2: every chain stops every step) with the parallel and the serial redo.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05d_parity.log 2>&1
rc=$?; tail -5 gpurun_out/r05d_parity.log; [ $rc -eq 0 ] || exit $rc
tools/ab_bench.sh r05d64 3 "--steps 400 --warmup 40" prod base || exit 1
tools/ab_bench.sh r05d8 3 "--steps 400 --warmup 40 --batch 8" prod base || exit 1
tools/ab_bench.sh r05dstop 1 "--steps 100 --warmup 20 --tv-tol 0.2" prod || exit 1
tools/ab_bench.sh r05dstop8 1 "--steps 100 --warmup 20 --tv-tol 0.2 --batch 8" prod || exit 1
timeout -k 10 300 python3 bench.py --no-cpu --steps 10 --warmup 4 --warmup-seconds 0.1 --tv-tol 0.2 --serial-redo > gpurun_out/r05d_serial64.json && tail -c 400 gpurun_out/r05d_serial64.json
