#!/bin/bash
# A/B of diagnostic builds (exp_libs/lib_NAME.so) within one GPU call, alternating, REPS rounds.
# Usage: tools/ab_libs.sh REPS "bench args" name1 name2 ...   (name "base:ARGS" = product lib with ARGS)
set -o pipefail
cd "$(dirname "$0")/.."
reps=$1; shift
bargs=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq 1 "$reps"); do
  for n in "$@"; do
    lib=exp_libs/lib_$n.so
    timeout -k 10 150 env PSGLA_LIB=$lib python3 bench.py --no-cpu --steps 200 --warmup 10 $bargs > gpurun_out/ab/$n.json || exit 1
    python3 - "$n" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab/{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:>12s} step {d['ms_per_step']:.4f} ms  kernel {d['roofline']['kernel_ms']:.5f} ms  isolated {d['roofline']['kernel_ms_isolated']:.5f}  frac {d['roofline']['frac']:.4f}", flush=True)
PY
  done
done
