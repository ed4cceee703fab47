#!/bin/bash
# round 5 call g: tile-kernel per-phase budgets on the exact one-workgroup-per-tile grid (diagnostic build
# exp_libs/lib_tdiag.so from tools/patches/tile_phasediag.py)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
: > gpurun_out/r05g_tile_phases.txt
for shape in "1 481 321" "1 321 481" "8 256 256" "16 256 256" "2 481 321"; do
  PSGLA_LIB=exp_libs/lib_tdiag.so timeout -k 10 120 python3 tools/tile_phasediag.py $shape >> gpurun_out/r05g_tile_phases.txt 2>&1 \
    || { tail -20 gpurun_out/r05g_tile_phases.txt; exit 1; }
done
grep -v "amdgpu.ids" gpurun_out/r05g_tile_phases.txt | grep -v '^{'
