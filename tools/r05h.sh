#!/bin/bash
# round 5 call h: deepinv's early stop forced on every chain every step (tol 0.2) in the product library --
# the row stream's parallel redo (64 chains) and the tile kernel's serial recompute (8 chains, castle batch 1),
# each beside the normal step (tol 1e-5) in the same call.  columns: tag | chains | HxW | tol | ms_per_step | kernel
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for cfg in "64 256 256" "8 256 256" "1 481 321"; do
  set -- $cfg
  for tol in 1e-5 0.2; do
    timeout -k 10 240 python3 bench.py --no-cpu --steps 200 --warmup 20 --batch $1 --H $2 --W $3 --tv-tol $tol \
      > gpurun_out/r05h_$1_$tol.json 2> gpurun_out/r05h_$1_$tol.err || { tail -20 gpurun_out/r05h_$1_$tol.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('gpurun_out/r05h_$1_$tol.json').read().strip().splitlines()[-1])
print('r05h |', $1, '| $2x$3 |', '$tol', '|', d['ms_per_step'], '|', d['roofline']['kernel'])"
  done
done
