#!/bin/bash
# Round 4, call b: the phase-unrolled front / back with cached segment geometry (exp_libs/lib_fb.so) --
# full GPU suite on it, per-step barrier diagnostic, interleaved A/B against the product library at the bench
# shape and the two real shapes at 64 chains.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in fb r0; do
  PSGLA_LIB=exp_libs/lib_$v.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "stream or fused or tile_kernel_equals or early_stop or smoke or cli_castle" > gpurun_out/r04b_${v}_tests.log 2>&1 \
    || { tail -30 gpurun_out/r04b_${v}_tests.log; exit 1; }
  tail -2 gpurun_out/r04b_${v}_tests.log
done
PSGLA_LIB=exp_libs/lib_sdiag3.so timeout -k 10 120 python3 tools/stream_stepdiag.py 64 > gpurun_out/r04b_stepdiag_r0.txt 2>&1 || exit 1
cat gpurun_out/r04b_stepdiag_r0.txt
tools/ab_bench.sh fb64 3 "--steps 400 --warmup 40" prod fb r0 || exit 1
tools/ab_bench.sh fb321 2 "--steps 100 --warmup 10 --warmup-seconds 0.5 --H 321 --W 481" prod fb r0 || exit 1
tools/ab_bench.sh fb481 2 "--steps 100 --warmup 10 --warmup-seconds 0.5 --H 481 --W 321" prod fb r0 || exit 1
