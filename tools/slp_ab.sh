#!/bin/bash
# Bitwise digest + timing A/B of two builds (exp_libs/lib_<a>.so vs lib_<b>.so) at 8 and 64 chains.
cd "$(dirname "$0")/.."
for v in "$@"; do PSGLA_LIB=exp_libs/lib_$v.so timeout -k 10 120 python3 tools/fast_digest.py 2>/dev/null || exit 1; done
for rep in 1 2; do
  for b in 8 64; do
    for v in "$@"; do
      r=$(PSGLA_LIB=exp_libs/lib_$v.so timeout -k 10 120 python3 -u bench.py --steps 200 --warmup 20 --batch $b --no-cpu --kernel-iters 3 --warmup-seconds 0.5 2>/dev/null | tail -1) || { echo "FAIL $v"; exit 1; }
      echo "$v $b $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel"], d["ms_per_step"], d["roofline"]["kernel_ms"])')"
    done
  done
done
