#!/bin/bash
# A/B of the product library against exp_libs/lib_<tag>.so on the tile-kernel shapes (3 alternations).
# One line per run: bench args | library | ms per step | kernel ms (HIP events) | kernel
cd /root/repo
run() {
  local v=$1; shift
  local r
  if [ "$v" = "prod" ]; then
    r=$(timeout -k 10 120 python3 bench.py --no-cpu --steps 300 --warmup 20 --warmup-seconds 0.3 "$@" 2>/dev/null | tail -1) || exit 1
  else
    r=$(PSGLA_LIB=exp_libs/lib_$v.so timeout -k 10 120 python3 bench.py --no-cpu --steps 300 --warmup 20 --warmup-seconds 0.3 "$@" 2>/dev/null | tail -1) || exit 1
  fi
  echo "$* | $v | $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["kernel"])')"
}
for rep in 1 2 3; do
  for v in "$@"; do
    run $v --batch 8; run $v --batch 16; run $v --batch 1 --H 481 --W 321; run $v --batch 1
  done
done
