#!/bin/bash
# round 5 call j: the parallel early-stop redo with its pending flag in the step's flag word (no load of its own),
# in both the row stream and the tile kernel.  The full GPU suite, then interleaved A/Bs against the library
# before the tile kernel's parallel redo (exp_libs/lib_base.so: 8fd98e3 sources), then the forced stop (tol 0.2).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r05j_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r05j_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r05j_gpu_tests.log
tools/ab_bench.sh r05j8 3 "--steps 400 --warmup 40 --batch 8" prod base || exit 1
tools/ab_bench.sh r05jc 3 "--steps 400 --warmup 40 --batch 1 --H 481 --W 321" prod base || exit 1
tools/ab_bench.sh r05j16 2 "--steps 400 --warmup 40 --batch 16" prod base || exit 1
tools/ab_bench.sh r05j64 3 "--steps 400 --warmup 40" prod base || exit 1
tools/ab_bench.sh r05jstop 1 "--steps 200 --warmup 20 --batch 8 --tv-tol 0.2" prod || exit 1
tools/ab_bench.sh r05jstopc 1 "--steps 200 --warmup 20 --batch 1 --H 481 --W 321 --tv-tol 0.2" prod || exit 1
tools/ab_bench.sh r05jstop64 1 "--steps 200 --warmup 20 --tv-tol 0.2" prod || exit 1
