#!/bin/bash
# Round-3 profile at a commit: the default bench (64 chains, stream kernel) and the 8-chain strong-scaling
# step (tile kernel): kernel-trace stats + PMC; the 1-GPU strong sweep with the driver's command; the default
# bench line (CPU baseline included).  Usage: tools/r03_prof.sh TAG COMMIT
set -o pipefail
cd "$(dirname "$0")/.."
T=${1:-r03a}
C=${2:-unknown}
tools/profile_round.sh ${T}64 $C tv_stream_kernel 64 > gpurun_out/prof64.log 2>&1 || { tail -20 gpurun_out/prof64.log; exit 1; }
tools/profile_round.sh ${T}8 $C tv_tile_kernel 8 > gpurun_out/prof8.log 2>&1 || { tail -20 gpurun_out/prof8.log; exit 1; }
tools/bench_sweep.sh gpurun_out/${T}_sweep.jsonl > /dev/null || exit 1
python3 -c "
import json
for l in open('gpurun_out/${T}_sweep.jsonl'):
    d = json.loads(l); print(d['config']['chains_per_gpu'], d['roofline']['kernel'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python3 bench.py > gpurun_out/${T}_bench.json || exit 1
tail -c 600 gpurun_out/${T}_bench.json
