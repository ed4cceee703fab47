#!/bin/bash
# Round 5, call e: the parallel early-stop redo of the stream kernel as its own kernel after each step (prod) vs
# inlined ahead of the next step's main pass (v0) vs the library before it (base): early-stop parity of prod,
# the step A/B at 64 / 8 chains, and a forced-stop run (tol 0.2: every chain stops every step).
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "early_stop or redo" > gpurun_out/r05e_parity.log 2>&1
rc=$?; tail -3 gpurun_out/r05e_parity.log; [ $rc -eq 0 ] || exit $rc
tools/ab_bench.sh r05e64 3 "--steps 400 --warmup 40" prod v0 base || exit 1
tools/ab_bench.sh r05e8 2 "--steps 400 --warmup 40 --batch 8" prod base || exit 1
tools/ab_bench.sh r05estop 1 "--steps 100 --warmup 20 --tv-tol 0.2" prod v0 || exit 1
