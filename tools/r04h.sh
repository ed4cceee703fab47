#!/bin/bash
# Round 4, call h: where the 64-chain stream step goes -- timing-only variants (wrong samples): no noise in the
# front; no wait for the front's LDS-DMA loads.
set -o pipefail
cd "$(dirname "$0")/.."
tools/ab_bench.sh h64 3 "--steps 400 --warmup 40" prod nonoise nowait || exit 1
