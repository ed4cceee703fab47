#!/bin/bash
# Compiler scheduling strategies (-mllvm -amdgpu-sched-strategy=...): bitwise digest of each build, then
# A/B at 64 chains (stream kernel) and 8 chains (tile kernel).
set -o pipefail
cd "$(dirname "$0")/.."
for v in base ilp memc iterilp; do
  echo "$v $(PSGLA_LIB=exp_libs/lib_$v.so timeout -k 10 120 python3 tools/fast_digest.py 2>/dev/null | tail -1)" || exit 1
done
tools/ab_libs.sh 2 "" base ilp memc iterilp 2>&1 | grep -v amdgpu.ids
tools/ab_libs.sh 2 "--batch 8" base ilp iterilp 2>&1 | grep -v amdgpu.ids
