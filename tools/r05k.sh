#!/bin/bash
# round 5 call k (diagnostic): the 72-row tile's exact parity with the pending-redo flag in the flag word (prod) or
# in redo[0] (exp_libs/lib_redo0.so), each twice
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in 1; do
  for lib in redo0b redo0; do
    if [ $lib = prod ]; then E=""; else E="PSGLA_LIB=exp_libs/lib_$lib.so"; fi
    env $E timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread \
      -k "test_tile_kernel_exact_vs_oracle and (24-130 or 24-100 or 12-100 or 24-40)" > gpurun_out/r05k_${lib}_$rep.log 2>&1
    echo "$lib $rep rc=$? $(tail -1 gpurun_out/r05k_${lib}_$rep.log)"
  done
done
