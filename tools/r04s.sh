#!/bin/bash
# Round 4, call s: kernel-trace + PMC profiles of the reference's real shape (castle 481 x 321): the row stream at 64
# chains (half-wave windows) and the tile kernel at batch 1 (the CLI default).
set -o pipefail
cd "$(dirname "$0")/.."
C=${1:-unknown}
tools/profile_round.sh r04s_c64 $C tv_stream_kernel 64 --H 481 --W 321 > gpurun_out/r04s_c64.log 2>&1 || { tail -20 gpurun_out/r04s_c64.log; exit 1; }
tools/profile_round.sh r04s_c1 $C tv_tile_kernel 1 --H 481 --W 321 > gpurun_out/r04s_c1.log 2>&1 || { tail -20 gpurun_out/r04s_c1.log; exit 1; }
python3 - <<'PY'
import json
for t in ("r04s_c64", "r04s_c1"):
    d = json.load(open(f"gpurun_out/prof_{t}/pmc.json"))
    print(t, d["kernel"], round(d["hbm_bytes_per_launch"] / 1e6, 2), "MB", {k: round(v, 3) for k, v in d["wave_cycle_split"].items()})
PY
