#!/bin/bash
# Round-4 final call at a commit: the full GPU suite, the closing measurements (tools/r04_final.sh), and the three DNN
# configurations.  Usage: tools/r04_close.sh TAG COMMIT
set -o pipefail
cd "$(dirname "$0")/.."
T=${1:-r04y}
C=${2:-unknown}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 \
  || { tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
tools/r04_final.sh $T $C || exit 1
: > gpurun_out/${T}_dnn.jsonl
for w in dncnn-inpaint dncnn-deblur drunet-ula; do
  timeout -k 10 300 python3 tools/bench_dnn.py --workload $w --channels-last >> gpurun_out/${T}_dnn.jsonl || exit 1
done
cat gpurun_out/${T}_dnn.jsonl
