#!/bin/bash
# A/B of the tile kernel's wave count (round 3): product library (72-row 8-wave tiles where 48-row tiles need
# two rounds), lib_nw8 (32/48-row tiles as 8 waves x 4/6 rows) and lib_no9 (the rule without 72-row tiles).
# One line per run: config, library, ms per step, kernel ms (HIP events).  Usage: tools/tile_nw_ab.sh [libs...]
cd /root/repo
run() {  # $1 = lib tag (prod: the product library), rest = bench args
  local v=$1; shift
  local r
  if [ "$v" = "prod" ]; then
    r=$(timeout -k 10 120 python3 bench.py --no-cpu --steps 200 --warmup 20 --warmup-seconds 0.3 "$@" 2>/dev/null | tail -1) || exit 1
  else
    r=$(PSGLA_LIB=exp_libs/lib_$v.so timeout -k 10 120 python3 bench.py --no-cpu --steps 200 --warmup 20 --warmup-seconds 0.3 "$@" 2>/dev/null | tail -1) || exit 1
  fi
  echo "$* | $v | $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["kernel"])')"
}
for rep in 1 2; do
  for v in "$@"; do
    run $v --batch 8; run $v --batch 16; run $v --batch 12; run $v --batch 1 --H 481 --W 321
    run $v --batch 1; run $v --batch 4 --H 481 --W 321
  done
done
