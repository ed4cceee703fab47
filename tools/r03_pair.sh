#!/bin/bash
# Row-pair kernel: parity tests, then pair vs stream bench (64 chains).
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pair" > $out/r03d_pair_tests.log 2>&1
rc=$?
tail -5 $out/r03d_pair_tests.log
[ $rc -ne 0 ] && { grep -m5 -B5 "Error\|assert" $out/r03d_pair_tests.log | head -40; exit 1; }
for v in pair stream pair stream; do
  timeout -k 10 150 python bench.py --steps 200 --warmup 20 --no-cpu --variant $v > $out/r03d_bench_$v.json 2> $out/r03d_bench_$v.err || { echo "bench $v failed"; tail -20 $out/r03d_bench_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/r03d_bench_$v.json')); print('$v', d['roofline']['kernel'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['kernel_ms_isolated'], d['roofline']['frac'], d['mmse_psnr_mean_db'])"
done
