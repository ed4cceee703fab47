#!/bin/bash
# Round 4, call d: the tile-kernel rules whose round-3 A/B crossed calls, re-run with every leg in ONE call and
# stderr kept: 72-row tiles (product) vs none (no9) vs 8-wave 32/48-row tiles (nw8) at
# B = 8 / 12 / 16 (256 x 256) and 481 x 321 at B = 1 / 4; the norm-copies rule (product: 8 copies where >= 128
# tiles share a chain) vs one copy (nc1) on castle B = 1, 321 x 481 B = 1 / 2 and 8 chains.
set -o pipefail
cd "$(dirname "$0")/.."
A="--steps 200 --warmup 20 --warmup-seconds 0.3"
for b in 8 12 16; do tools/ab_bench.sh d_nw_b$b 3 "$A --batch $b" prod no9 nw8 || exit 1; done
tools/ab_bench.sh d_nw_castle1 3 "$A --batch 1 --H 481 --W 321" prod no9 nw8 || exit 1
tools/ab_bench.sh d_nw_castle4 3 "$A --batch 4 --H 481 --W 321" prod no9 nw8 || exit 1
tools/ab_bench.sh d_nc_castle1 3 "$A --batch 1 --H 481 --W 321" prod nc1 || exit 1
tools/ab_bench.sh d_nc_321b1 3 "$A --batch 1 --H 321 --W 481" prod nc1 || exit 1
tools/ab_bench.sh d_nc_321b2 3 "$A --batch 2 --H 321 --W 481" prod nc1 || exit 1
tools/ab_bench.sh d_nc_b8 3 "$A --batch 8" prod nc1 || exit 1
