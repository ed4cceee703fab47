#!/bin/bash
# Small-batch probe: band kernel vs stream kernel (row-split counts) at 8 / 16 / 64 chains.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r02b
mkdir -p $O
: > $O/probe.jsonl
run() { timeout -k 10 120 python3 bench.py --steps 100 --warmup 10 --warmup-seconds 0.5 --no-cpu "$@" >> $O/probe.jsonl; }
run --batch 8 --variant band &&
run --batch 16 --variant band &&
run --batch 64 --variant band &&
run --batch 8 --stream-wgs 128 &&
run --batch 8 --stream-wgs 64 &&
run --batch 8 &&
run --batch 64
