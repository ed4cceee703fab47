#!/bin/bash
# A/B of the barrier and P2P stream pipelines in one call (alternating), plus the P2P parity tests.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/ab_p2p
mkdir -p $O
: > $O/ab.jsonl
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k p2p > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for v in stream p2p; do
    timeout -k 10 200 python3 bench.py --steps 200 --warmup 10 --no-cpu --variant $v "$@" >> $O/ab.jsonl || exit 1
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/ab_p2p/ab.jsonl"):
    d = json.loads(l)
    print(d["config"]["chains_per_gpu"], d["roofline"]["kernel"], d["ms_per_step"], d["roofline"]["kernel_ms_isolated"], d["roofline"]["frac"])
PY
