#!/bin/bash
# Round 4, call e: the product library with the round-4 stream kernel (phase-unrolled front / back, cached
# segment geometry, no ring 0 at alpha = 1, half-wave windows for 256 < W <= 324): full GPU suite, per-step
# barrier diagnostic, interleaved A/B against the round-start stream kernel (base) and fb at the bench shape and
# both real orientations at 64 chains; then the tile-rule A/Bs (tools/r04d.sh).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
tools/gpu_tests.sh > /dev/null || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
PSGLA_LIB=exp_libs/lib_sdiag4.so timeout -k 10 120 python3 tools/stream_stepdiag.py 64 > gpurun_out/r04e_stepdiag.txt 2>&1 || { cat gpurun_out/r04e_stepdiag.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04e_stepdiag.txt
tools/ab_bench.sh e64 3 "--steps 400 --warmup 40" base fb prod || exit 1
tools/ab_bench.sh e321 2 "--steps 100 --warmup 10 --warmup-seconds 0.5 --H 321 --W 481" base fb prod || exit 1
tools/ab_bench.sh e481w 2 "--steps 100 --warmup 10 --warmup-seconds 0.5 --H 481 --W 321 --stream-windows whole" base fb prod || exit 1
tools/ab_bench.sh e481 2 "--steps 100 --warmup 10 --warmup-seconds 0.5 --H 481 --W 321" prod || exit 1
tools/r04d.sh
