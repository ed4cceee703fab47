#!/bin/bash
# Round 5, call c: ablations of the classic row stream at 64 chains (timing-only builds, kernel_ms_isolated =
# main pass only): no noise, no front DMA, no back DMA, no stores, no stage rings.
set -o pipefail
cd "$(dirname "$0")/.."
tools/ab_bench.sh r05c 2 "--steps 200 --warmup 20" prod nonoise nofdma nobdma nostore noring
