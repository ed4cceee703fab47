#!/bin/bash
cd /root/repo
for args in "--batch 1 --H 481 --W 321 --variant tile" "--batch 1 --H 321 --W 481 --variant tile" "--batch 1 --variant tile" "--batch 2 --H 481 --W 321 --variant tile" "--batch 4 --variant tile"; do
  for v in none r2 none r2; do
    r=$(PSGLA_LIB=exp_libs/lib_$v.so timeout -k 10 120 python3 bench.py --no-cpu --steps 200 --warmup 20 --warmup-seconds 0.3 $args 2>/dev/null | tail -1) || exit 1
    echo "$args $v $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"])')"
  done
done
