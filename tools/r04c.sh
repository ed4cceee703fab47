#!/bin/bash
# Round 4, call c: stream kernel variants -- r0 (phase-unrolled front / back + no ring 0: stage 1 reads the
# front's staging) parity tests; per-step barrier diagnostics of the committed kernel, fb and r0; interleaved
# A/B prod / fb / r0 at the bench shape and the two real shapes at 64 chains.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
PSGLA_LIB=exp_libs/lib_r0.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04c_r0_tests.log 2>&1 || { tail -30 gpurun_out/r04c_r0_tests.log; exit 1; }
tail -2 gpurun_out/r04c_r0_tests.log
for v in sdiagb sdiagfb sdiag3; do
  echo "== $v"
  PSGLA_LIB=exp_libs/lib_$v.so timeout -k 10 120 python3 tools/stream_stepdiag.py 64 > gpurun_out/r04c_stepdiag_$v.txt 2>&1 || { cat gpurun_out/r04c_stepdiag_$v.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r04c_stepdiag_$v.txt
done
tools/ab_bench.sh c64 3 "--steps 400 --warmup 40" prod fb r0 || exit 1
tools/ab_bench.sh c321 2 "--steps 100 --warmup 10 --warmup-seconds 0.5 --H 321 --W 481" prod fb r0 || exit 1
tools/ab_bench.sh c481 2 "--steps 100 --warmup 10 --warmup-seconds 0.5 --H 481 --W 321" prod fb r0 || exit 1
