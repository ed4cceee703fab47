#!/bin/bash
cd /root/repo
for args in "--batch 1 --H 481 --W 256 --variant tile" "--batch 1 --H 481 --W 256 --variant stream" "--batch 1 --H 481 --W 320 --variant stream" "--batch 1 --H 481 --W 321" "--batch 2 --H 481 --W 256 --variant tile" "--batch 1 --H 321 --W 481" "--batch 1 --H 256 --W 256 --variant tile" "--batch 1 --H 256 --W 256 --variant stream"; do
  r=$(timeout -k 10 120 python3 bench.py --no-cpu --steps 200 --warmup 20 --warmup-seconds 0.5 $args | tail -1) || exit 1
  echo "$args => $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel"], d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
