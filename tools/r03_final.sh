#!/bin/bash
# Round-3 closing measurements at a commit: stream (64) / tile (8) kernel-trace + PMC profiles, the one-GPU
# strong sweep, the default bench line, castle timing (B = 1 tile, B = 64 stream), the DNN configurations.
# Usage: tools/r03_final.sh TAG COMMIT
set -o pipefail
cd "$(dirname "$0")/.."
T=${1:-r03b}
C=${2:-unknown}
tools/r03_prof.sh $T $C || exit 1
timeout -k 10 300 python3 tools/castle_timing.py 10000 1 > gpurun_out/${T}_castle_b1.json || exit 1
timeout -k 10 300 python3 tools/castle_timing.py 2000 64 > gpurun_out/${T}_castle_b64.json || exit 1
cat gpurun_out/${T}_castle_b1.json gpurun_out/${T}_castle_b64.json
: > gpurun_out/${T}_dnn.jsonl
for w in dncnn-inpaint dncnn-deblur drunet-ula; do
  timeout -k 10 300 python3 tools/bench_dnn.py --workload $w --channels-last >> gpurun_out/${T}_dnn.jsonl || exit 1
done
cat gpurun_out/${T}_dnn.jsonl
