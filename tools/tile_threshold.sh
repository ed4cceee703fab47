#!/bin/bash
# Tile vs stream kernel around the auto-dispatch threshold (tiles <= CUs): forced variants, bench step.
cd "$(dirname "$0")/.."
for shape in "--H 481 --W 321" "--H 321 --W 481" "--H 256 --W 256"; do
  for b in 3 4 6 8 12 16; do
    for v in tile stream; do
      r=$(timeout -k 10 120 python3 bench.py --no-cpu --steps 200 --warmup 20 --warmup-seconds 0.3 --batch $b $shape --variant $v 2>/dev/null | tail -1) || exit 1
      echo "$shape B=$b $v $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
    done
  done
done
