#!/bin/bash
# Closing profile part 2 (one GPU call): castle timing in both orientations at batch 1 and 64, the tile kernel's
# per-phase budget (when exp_libs/lib_tdiag.so exists), the DNN configurations' bench lines and HIP-pass kernel traces.
# Usage: tools/close_part2.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
T=${1:?tag}
mkdir -p gpurun_out
: > gpurun_out/${T}_castle.jsonl
for args in "10000 1" "10000 1 T" "2000 64" "2000 64 T"; do
  timeout -k 10 300 python3 tools/castle_timing.py $args >> gpurun_out/${T}_castle.jsonl || exit 1
done
cat gpurun_out/${T}_castle.jsonl
if [ -f exp_libs/lib_tdiag.so ]; then
  : > gpurun_out/${T}_tile_phases.txt
  for shape in "8 256 256" "16 256 256" "1 481 321" "1 321 481"; do
    PSGLA_LIB=exp_libs/lib_tdiag.so timeout -k 10 120 python3 tools/tile_phasediag.py $shape >> gpurun_out/${T}_tile_phases.txt 2>&1 \
      || { tail -20 gpurun_out/${T}_tile_phases.txt; exit 1; }
  done
  grep -v "amdgpu.ids" gpurun_out/${T}_tile_phases.txt | tail -40
fi
tools/dnn_prof.sh ${T} || exit 1
cat gpurun_out/${T}_dnn_bench.jsonl
