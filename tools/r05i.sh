#!/bin/bash
# round 5 call i: the tile kernel's parallel early-stop redo.  Parity (the early-stop / redo / hand-off GPU tests),
# then interleaved A/Bs against the library before it (exp_libs/lib_base.so: serial recompute, 8fd98e3 sources),
# then the forced stop (tol 0.2) in the product.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "early_stop or redo or handoff or tile" > gpurun_out/r05i_parity.log 2>&1 || { tail -40 gpurun_out/r05i_parity.log; exit 1; }
tail -1 gpurun_out/r05i_parity.log
tools/ab_bench.sh r05i8 3 "--steps 400 --warmup 40 --batch 8" prod base || exit 1
tools/ab_bench.sh r05ic 3 "--steps 400 --warmup 40 --batch 1 --H 481 --W 321" prod base || exit 1
tools/ab_bench.sh r05i16 2 "--steps 400 --warmup 40 --batch 16" prod base || exit 1
tools/ab_bench.sh r05i64 2 "--steps 400 --warmup 40" prod base || exit 1
tools/ab_bench.sh r05istop 1 "--steps 200 --warmup 20 --batch 8 --tv-tol 0.2" prod || exit 1
tools/ab_bench.sh r05istopc 1 "--steps 200 --warmup 20 --batch 1 --H 481 --W 321 --tv-tol 0.2" prod || exit 1
