#!/bin/bash
# A/B of multi-step tile kernel diagnostic builds (exp_libs/lib_<name>.so) at 8 chains, one call.
# A name ending in "+single" runs that build with one tile-kernel launch per step (bench default).
cd "$(dirname "$0")/.."
for rep in 1 2; do
  for v in "$@"; do
    lib=${v%+single}; extra="--multi-step"; [ "$lib" != "$v" ] && extra=""
    r=$(PSGLA_LIB=exp_libs/lib_$lib.so timeout -k 10 120 python3 -u bench.py --steps 200 --warmup 20 --batch 8 --no-cpu --kernel-iters 3 --warmup-seconds 0.5 $extra 2>/dev/null | tail -1) || { echo "FAIL $v"; exit 1; }
    echo "$v $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel"], d["ms_per_step"], d["roofline"]["kernel_ms"])')"
  done
done
