#!/bin/bash
# Round 4, call l: the tile kernel's rel-err sums spread over waves (product) against all on wave 0 (redw0); eight
# norm copies from 64 tiles per chain (product) against from 128 (nc128); tile parity tests; per-phase budget.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "tile or early_stop or fused or castle" \
  > gpurun_out/r04l_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r04l_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04l_gpu_tests.log
tools/ab_bench.sh l8 4 "--steps 400 --warmup 40 --warmup-seconds 0.5 --batch 8" prod redw0 || exit 1
tools/ab_bench.sh l16 3 "--steps 200 --warmup 20 --warmup-seconds 0.5 --batch 16" prod redw0 || exit 1
tools/ab_bench.sh lc1 3 "--steps 400 --warmup 40 --warmup-seconds 0.5 --batch 1 --H 481 --W 321" prod redw0 || exit 1
tools/ab_bench.sh lb1 3 "--steps 400 --warmup 40 --warmup-seconds 0.5 --batch 1" prod nc128 || exit 1
tools/ab_bench.sh lb2 3 "--steps 400 --warmup 40 --warmup-seconds 0.5 --batch 2" prod nc128 || exit 1
tools/ab_bench.sh lc2 3 "--steps 400 --warmup 40 --warmup-seconds 0.5 --batch 2 --H 481 --W 321" prod nc128 || exit 1
: > gpurun_out/r04l_tile_phases.txt
for shape in "8 256 256" "1 481 321"; do
  PSGLA_LIB=exp_libs/lib_tdiag.so timeout -k 10 120 python3 tools/tile_phasediag.py $shape >> gpurun_out/r04l_tile_phases.txt 2>&1 \
    || { tail -20 gpurun_out/r04l_tile_phases.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/r04l_tile_phases.txt | grep -v "^{"
