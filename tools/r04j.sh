#!/bin/bash
# Round 4, call j: the tile kernel's mean / sq DMA deferred past the data term (product) against the round-4 tile
# kernel that issues it with the other loads (mstearly): tile parity tests, interleaved A/B at 8 chains (the 8-GPU
# strong-scaling point), castle at batch 1 and 4, 16 chains (72-row tiles), and the per-phase budget of the product.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "tile or early_stop or fused" \
  > gpurun_out/r04j_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r04j_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04j_gpu_tests.log
tools/ab_bench.sh j8 4 "--steps 400 --warmup 40 --warmup-seconds 0.5 --batch 8" prod mstearly || exit 1
tools/ab_bench.sh jc1 3 "--steps 400 --warmup 40 --warmup-seconds 0.5 --batch 1 --H 481 --W 321" prod mstearly || exit 1
tools/ab_bench.sh jc4 3 "--steps 200 --warmup 20 --warmup-seconds 0.5 --batch 4 --H 481 --W 321" prod mstearly || exit 1
tools/ab_bench.sh j16 3 "--steps 200 --warmup 20 --warmup-seconds 0.5 --batch 16" prod mstearly || exit 1
for shape in "8 256 256" "1 481 321"; do
  PSGLA_LIB=exp_libs/lib_tdiag.so timeout -k 10 120 python3 tools/tile_phasediag.py $shape >> gpurun_out/r04j_tile_phases.txt 2>&1 \
    || { tail -20 gpurun_out/r04j_tile_phases.txt; exit 1; }
done
cat gpurun_out/r04j_tile_phases.txt
