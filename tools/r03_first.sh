#!/bin/bash
# Round 3, first GPU look at the row-pair kernel: bench stream vs pair (64 chains), then the pair tests.
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out
for v in pair stream pair stream; do
  timeout -k 10 150 python bench.py --steps 200 --warmup 20 --no-cpu --variant $v > $out/r03a_bench_$v.json 2> $out/r03a_bench_$v.err || { echo "bench $v failed"; tail -20 $out/r03a_bench_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$out/r03a_bench_$v.json')); print('$v', d['roofline']['kernel'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['kernel_ms_isolated'], d['roofline']['frac'], d['mmse_psnr_mean_db'])" | tee -a $out/r03a_summary.txt
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pair" > $out/r03a_pair_tests.log 2>&1
rc=$?
tail -30 $out/r03a_pair_tests.log
exit $rc
