#!/bin/bash
# round 5 call m: cost of the tile kernel's parallel redo on normal steps -- prod (pending word loaded in the redo
# branch), hoist (loaded at kernel entry; timing only, fast mode), base (serial recompute, 8fd98e3 sources)
set -o pipefail
cd "$(dirname "$0")/.."
tools/ab_bench.sh r05m8 4 "--steps 400 --warmup 40 --batch 8" prod hoist base || exit 1
tools/ab_bench.sh r05mc 4 "--steps 400 --warmup 40 --batch 1 --H 481 --W 321" prod hoist base || exit 1
tools/ab_bench.sh r05m16 2 "--steps 400 --warmup 40 --batch 16" prod hoist base || exit 1
tools/ab_bench.sh r05mstop 1 "--steps 200 --warmup 20 --batch 8 --tv-tol 0.2" prod || exit 1
tools/ab_bench.sh r05mstopc 1 "--steps 200 --warmup 20 --batch 1 --H 481 --W 321 --tv-tol 0.2" prod || exit 1
tools/ab_bench.sh r05mstop16 1 "--steps 200 --warmup 20 --batch 16 --tv-tol 0.2" prod || exit 1
