#!/bin/bash
# Round 4, call a: the product library after the translation-unit split (ABI 9) -- full GPU suite, default
# bench line, per-step barrier diagnostic of the stream kernel; the tile kernel's u2 store A/B (timing + HBM
# bytes); then call b (tools/r04b.sh: the phase-unrolled front / back).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
tools/gpu_tests.sh > /dev/null || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python3 bench.py > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || { tail gpurun_out/r04a_bench.err; exit 1; }
tail -1 gpurun_out/r04a_bench.json
timeout -k 10 120 python3 tools/stream_stepdiag.py 64 > gpurun_out/r04a_stepdiag.txt 2>&1 || { cat gpurun_out/r04a_stepdiag.txt; exit 1; }
cat gpurun_out/r04a_stepdiag.txt
tools/ab_bench.sh u2 3 "--batch 8 --steps 200 --warmup 20 --warmup-seconds 0.3" prod u2old u2nt | tee gpurun_out/r04a_u2_ab.txt || exit 1
tools/ab_pmc.sh u2 tv_tile_kernel "--batch 8" prod u2old u2nt | tee gpurun_out/r04a_u2_pmc.txt || exit 1
tools/r04b.sh
