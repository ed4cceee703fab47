#!/bin/bash
# Round 4, call i: psgla noise v2 (row-aligned noise quads) -- the full GPU suite, then the interleaved A/B of the
# product against the same library with the round-4 v1 row-stream / tile kernels (lib_v1: two Philox per lane on
# W % 4 != 0 rows) at both castle orientations (64 chains) and castle batch 1 / 8; the tile kernel's per-phase
# budget; where the 64-chain stream step goes (timing-only variants: no noise, no front load wait).
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04i_gpu_tests.log 2>&1 \
  || { tail -30 gpurun_out/r04i_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04i_gpu_tests.log
tools/ab_bench.sh i481 3 "--steps 100 --warmup 10 --warmup-seconds 0.5 --H 481 --W 321" prod v1 || exit 1
tools/ab_bench.sh i321 3 "--steps 100 --warmup 10 --warmup-seconds 0.5 --H 321 --W 481" prod v1 || exit 1
tools/ab_bench.sh i481b1 3 "--steps 400 --warmup 40 --warmup-seconds 0.5 --batch 1 --H 481 --W 321" prod v1 || exit 1
tools/ab_bench.sh i481b8 3 "--steps 200 --warmup 20 --warmup-seconds 0.5 --batch 8 --H 481 --W 321" prod v1 || exit 1
for shape in "8 256 256" "1 481 321" "1 321 481"; do
  PSGLA_LIB=exp_libs/lib_tdiag.so timeout -k 10 120 python3 tools/tile_phasediag.py $shape >> gpurun_out/r04i_tile_phases.txt 2>&1 \
    || { tail -20 gpurun_out/r04i_tile_phases.txt; exit 1; }
done
cat gpurun_out/r04i_tile_phases.txt
tools/ab_bench.sh i64 3 "--steps 400 --warmup 40" prod nonoise nowait || exit 1
