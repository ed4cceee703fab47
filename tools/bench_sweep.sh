#!/bin/bash
# One-GPU strong-scaling ceiling: the bench step at 8/16/32/64 chains (64/N chains per GPU at N GPUs),
# each with the driver's step/warm-up counts.  Usage: tools/bench_sweep.sh OUTFILE [extra bench args]
set -e
cd "$(dirname "$0")/.."
OUT=${1:-gpurun_out/sweep.jsonl}
shift || true
: > $OUT
for b in 64 32 16 8; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu --batch $b "$@" >> $OUT
done
cat $OUT
