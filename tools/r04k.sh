#!/bin/bash
# Round 4, call k: the tile kernel's finaliser reads its norm copies back to back (product) against one round trip
# per copy (finser), and eight norm copies for every tile launch (nc8all); tile / early-stop parity tests; the
# per-phase budget of the product at castle batch 1.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "tile or early_stop or fused or castle" \
  > gpurun_out/r04k_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r04k_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04k_gpu_tests.log
tools/ab_bench.sh kc1 3 "--steps 400 --warmup 40 --warmup-seconds 0.5 --batch 1 --H 481 --W 321" prod finser nc8all || exit 1
tools/ab_bench.sh kt1 3 "--steps 400 --warmup 40 --warmup-seconds 0.5 --batch 1 --H 321 --W 481" prod finser nc8all || exit 1
tools/ab_bench.sh kc2 3 "--steps 400 --warmup 40 --warmup-seconds 0.5 --batch 2 --H 481 --W 321" prod finser nc8all || exit 1
tools/ab_bench.sh k8 3 "--steps 400 --warmup 40 --warmup-seconds 0.5 --batch 8" prod finser nc8all || exit 1
tools/ab_bench.sh k16 3 "--steps 200 --warmup 20 --warmup-seconds 0.5 --batch 16" prod finser nc8all || exit 1
: > gpurun_out/r04k_tile_phases.txt
for shape in "1 481 321" "8 256 256"; do
  PSGLA_LIB=exp_libs/lib_tdiag.so timeout -k 10 120 python3 tools/tile_phasediag.py $shape >> gpurun_out/r04k_tile_phases.txt 2>&1 \
    || { tail -20 gpurun_out/r04k_tile_phases.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/r04k_tile_phases.txt | grep -v "^{"
