#!/bin/bash
# Round 4, call g: what row-aligned noise quads would save on odd widths (timing-only variant esh0: its noise
# is wrong for W % 4 != 0) -- stream kernel at 64 chains both castle orientations, tile kernel at batch 1 / 8.
set -o pipefail
cd "$(dirname "$0")/.."
tools/ab_bench.sh g481 3 "--steps 100 --warmup 10 --warmup-seconds 0.5 --H 481 --W 321" prod esh0 || exit 1
tools/ab_bench.sh g321 3 "--steps 100 --warmup 10 --warmup-seconds 0.5 --H 321 --W 481" prod esh0 || exit 1
tools/ab_bench.sh g481b1 3 "--steps 400 --warmup 40 --warmup-seconds 0.5 --batch 1 --H 481 --W 321" prod esh0 || exit 1
tools/ab_bench.sh g481b8 3 "--steps 200 --warmup 20 --warmup-seconds 0.5 --batch 8 --H 481 --W 321" prod esh0 || exit 1
# per-phase budget of the tile kernel (diagnostic build; 8 chains of 256 x 256, castle at batch 1)
PSGLA_LIB=exp_libs/lib_tdiag.so timeout -k 10 120 python3 tools/tile_phasediag.py 8 256 256 > gpurun_out/r04g_tdiag8.txt 2>&1 || { tail -20 gpurun_out/r04g_tdiag8.txt; exit 1; }
PSGLA_LIB=exp_libs/lib_tdiag.so timeout -k 10 120 python3 tools/tile_phasediag.py 1 481 321 > gpurun_out/r04g_tdiagc.txt 2>&1 || { tail -20 gpurun_out/r04g_tdiagc.txt; exit 1; }
cat gpurun_out/r04g_tdiag8.txt gpurun_out/r04g_tdiagc.txt
