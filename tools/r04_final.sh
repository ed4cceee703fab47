#!/bin/bash
# Round-4 closing measurements at a commit: stream (64) / tile (8) kernel-trace + PMC profiles, the one-GPU strong
# sweep with the driver's command, the default bench line (its roofline.traffic from this call's PMC summary),
# castle timing in both orientations at batch 1 and 64, and the tile kernel's per-phase budget (diagnostic build
# lib_tdiag from the same sources).  Usage: tools/r04_final.sh TAG COMMIT
set -o pipefail
cd "$(dirname "$0")/.."
T=${1:-r04z}
C=${2:-unknown}
tools/profile_round.sh ${T}64 $C tv_stream_kernel 64 > gpurun_out/${T}_prof64.log 2>&1 || { tail -20 gpurun_out/${T}_prof64.log; exit 1; }
tools/profile_round.sh ${T}8 $C tv_tile_kernel 8 > gpurun_out/${T}_prof8.log 2>&1 || { tail -20 gpurun_out/${T}_prof8.log; exit 1; }
tools/bench_sweep.sh gpurun_out/${T}_sweep.jsonl > /dev/null || exit 1
python3 -c "
import json
for l in open('gpurun_out/${T}_sweep.jsonl'):
    d = json.loads(l); print(d['config']['chains_per_gpu'], d['roofline']['kernel'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python3 bench.py --pmc-json gpurun_out/prof_${T}64/pmc.json > gpurun_out/${T}_bench.json || exit 1
tail -c 900 gpurun_out/${T}_bench.json
: > gpurun_out/${T}_castle.jsonl
for args in "10000 1" "10000 1 T" "2000 64" "2000 64 T"; do
  timeout -k 10 300 python3 tools/castle_timing.py $args >> gpurun_out/${T}_castle.jsonl || exit 1
done
cat gpurun_out/${T}_castle.jsonl
: > gpurun_out/${T}_tile_phases.txt
for shape in "8 256 256" "1 481 321" "1 321 481"; do
  PSGLA_LIB=exp_libs/lib_tdiag.so timeout -k 10 120 python3 tools/tile_phasediag.py $shape >> gpurun_out/${T}_tile_phases.txt 2>&1 \
    || { tail -20 gpurun_out/${T}_tile_phases.txt; exit 1; }
done
grep -v "amdgpu.ids" gpurun_out/${T}_tile_phases.txt
