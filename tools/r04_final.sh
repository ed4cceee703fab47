#!/bin/bash
# Round-4 closing measurements at a commit: stream (64) / tile (8) kernel-trace + PMC profiles, the one-GPU strong
# sweep, the default bench line (tools/r03_prof.sh), castle timing in both orientations at batch 1 and 64, and the
# tile kernel's per-phase budget (diagnostic build lib_tdiag, rebuilt from the same sources).
# Usage: tools/r04_final.sh TAG COMMIT
set -o pipefail
cd "$(dirname "$0")/.."
T=${1:-r04z}
C=${2:-unknown}
tools/r03_prof.sh $T $C || exit 1
: > gpurun_out/${T}_castle.jsonl
for args in "10000 1" "10000 1 T" "2000 64" "2000 64 T"; do
  timeout -k 10 300 python3 tools/castle_timing.py $args >> gpurun_out/${T}_castle.jsonl || exit 1
done
cat gpurun_out/${T}_castle.jsonl
for shape in "8 256 256" "1 481 321" "1 321 481"; do
  PSGLA_LIB=exp_libs/lib_tdiag.so timeout -k 10 120 python3 tools/tile_phasediag.py $shape >> gpurun_out/${T}_tile_phases.txt 2>&1 \
    || { tail -20 gpurun_out/${T}_tile_phases.txt; exit 1; }
done
cat gpurun_out/${T}_tile_phases.txt
