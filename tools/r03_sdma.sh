#!/bin/bash
# Stage-1-issued front DMA (PSGLA_STAGE_DMA=1): stream parity tests on that build, then A/B vs base.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
PSGLA_LIB=exp_libs/lib_sdma.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "stream or fused or early_stop" > gpurun_out/r03h_sdma_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r03h_sdma_tests.log
[ $rc -ne 0 ] && { grep -m3 -A30 "^____" gpurun_out/r03h_sdma_tests.log | head -60; exit 1; }
tools/ab_libs.sh 3 "" base sdma
