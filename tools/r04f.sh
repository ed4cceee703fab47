#!/bin/bash
# Round 4, call f: the front's noise spread over its four phases (product) -- stream / fused parity tests, step
# diagnostic, interleaved A/B against d74b03e's stream kernel (r1) and the round-start kernel (base) at the bench
# shape and both real orientations (castle timing: tools/castle_timing.py); forced half-wave windows at 256 x 256
# (the halo cost of 128-column pipelines).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "stream or fused or tile_kernel_equals or early_stop or smoke or noise" > gpurun_out/r04f_tests.log 2>&1 \
  || { tail -30 gpurun_out/r04f_tests.log; exit 1; }
tail -2 gpurun_out/r04f_tests.log
PSGLA_LIB=exp_libs/lib_sdiag5.so timeout -k 10 120 python3 tools/stream_stepdiag.py 64 > gpurun_out/r04f_stepdiag.txt 2>&1 || { cat gpurun_out/r04f_stepdiag.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04f_stepdiag.txt
tools/ab_bench.sh f64 3 "--steps 400 --warmup 40" base r1 prod || exit 1
tools/ab_bench.sh f321 2 "--steps 100 --warmup 10 --warmup-seconds 0.5 --H 321 --W 481" r1 prod || exit 1
tools/ab_bench.sh f481 2 "--steps 100 --warmup 10 --warmup-seconds 0.5 --H 481 --W 321" r1 prod || exit 1
tools/ab_bench.sh f64half 1 "--steps 200 --warmup 20 --stream-windows half" prod || exit 1
