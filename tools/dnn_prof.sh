#!/bin/bash
# Kernel traces of the three DNN configurations (tools/bench_dnn.py at 64 x 3 x 256 x 256) and the achieved HBM
# bandwidth of their HIP passes (tools/dnn_pass_roofline.py).  Usage: tools/dnn_prof.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
T=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/${T}_dnn_passes.jsonl
: > gpurun_out/${T}_dnn_bench.jsonl
for w in dncnn-inpaint dncnn-deblur drunet-ula; do
  O=gpurun_out/prof_${T}_$w
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o p -- \
    python3 tools/bench_dnn.py --workload $w --channels-last > $O.bench.json || exit 1
  tail -1 $O.bench.json >> gpurun_out/${T}_dnn_bench.jsonl
  python3 tools/dnn_pass_roofline.py --workload $w --stats $O/p_kernel_stats.csv >> gpurun_out/${T}_dnn_passes.jsonl || exit 1
  cp $O/p_kernel_stats.csv gpurun_out/${T}_${w}_kernel_stats.csv
done
cat gpurun_out/${T}_dnn_passes.jsonl
