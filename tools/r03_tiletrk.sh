#!/bin/bash
# Tile kernel: tracked / untracked primal instantiations -- tile parity tests, then A/B vs HEAD at 8 chains
# and castle B = 1.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "tile or auto_dispatch" > gpurun_out/r03m_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r03m_tests.log
[ $rc -ne 0 ] && { grep -m3 -A40 "^____" gpurun_out/r03m_tests.log | head -80; exit 1; }
tools/ab_libs.sh 3 "--batch 8" head new
tools/ab_libs.sh 2 "--batch 1 --H 481 --W 321" head new
