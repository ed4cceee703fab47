#!/bin/bash
# Round 4, call q: round-end readiness at the final tree -- smoke(), the driver's bench command, one rocprofv3
# kernel-trace summary of it.
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r04q_bench.json || exit 1
tail -c 700 gpurun_out/r04q_bench.json
