#!/bin/bash
# Round-2 profile at a commit: default bench (64 chains, stream kernel) and the 8-chain strong-scaling
# step (tile kernel): kernel-trace stats + PMC; the 1-GPU strong sweep with the driver's command.
set -o pipefail
cd "$(dirname "$0")/.."
C=${1:-unknown}
tools/profile_round.sh r02e64 $C tv_stream_kernel 64 > gpurun_out/prof64.log 2>&1 || { tail -20 gpurun_out/prof64.log; exit 1; }
tools/profile_round.sh r02e8 $C tv_tile_kernel 8 > gpurun_out/prof8.log 2>&1 || { tail -20 gpurun_out/prof8.log; exit 1; }
tools/bench_sweep.sh gpurun_out/r02e_sweep.jsonl > /dev/null || exit 1
cat gpurun_out/r02e_sweep.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config']['chains_per_gpu'], d['roofline']['kernel'], d['ms_per_step'], d['roofline']['frac'])"
