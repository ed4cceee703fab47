#!/bin/bash
# Diagnostic timing builds of libpsgla_hip.so (never loaded by the product; bench.py picks one via
# PSGLA_LIB).  Usage: tools/build_variants.sh NAME "-DFLAG ..." [NAME "-DFLAG ..."]...
set -e
cd "$(dirname "$0")/.."
mkdir -p exp_libs
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -Wno-inline-asm \
    -fPIC -shared -I include $flags -o exp_libs/lib_$name.so psgla_for_posterior_sampling_amd/csrc/psgla_kernels.hip &
done
wait
ls -la exp_libs
