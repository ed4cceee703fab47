#!/bin/bash
# round 5 call l: the tile kernel's parallel early-stop redo (pending flag in redo[0], loaded in the redo branch:
# prod; loaded at kernel entry: exp_libs/lib_hoist.so).  The full GPU suite on prod, the tile / redo parity subset on
# hoist, interleaved A/Bs against the library before it (lib_base: 8fd98e3 sources), the forced stop (tol 0.2).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r05l_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r05l_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r05l_gpu_tests.log
PSGLA_LIB=exp_libs/lib_hoist.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "tile or redo or early_stop or handoff" > gpurun_out/r05l_hoist_parity.log 2>&1 \
  || { tail -40 gpurun_out/r05l_hoist_parity.log; exit 1; }
tail -1 gpurun_out/r05l_hoist_parity.log
tools/ab_bench.sh r05l8 3 "--steps 400 --warmup 40 --batch 8" prod hoist base || exit 1
tools/ab_bench.sh r05lc 3 "--steps 400 --warmup 40 --batch 1 --H 481 --W 321" prod hoist base || exit 1
tools/ab_bench.sh r05l16 2 "--steps 400 --warmup 40 --batch 16" prod hoist base || exit 1
tools/ab_bench.sh r05lstop 1 "--steps 200 --warmup 20 --batch 8 --tv-tol 0.2" prod hoist || exit 1
tools/ab_bench.sh r05lstopc 1 "--steps 200 --warmup 20 --batch 1 --H 481 --W 321 --tv-tol 0.2" prod hoist || exit 1
tools/ab_bench.sh r05lstop16 1 "--steps 200 --warmup 20 --batch 16 --tv-tol 0.2" prod hoist || exit 1
