#!/bin/bash
# A/B of diagnostic builds within one GPU call with extra bench arguments (e.g. --batch 8):
# tools/ab_args.sh REPS "bench args" name1 name2 ...
set -e
cd "$(dirname "$0")/.."
reps=$1; shift
args=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 "$reps"); do
  for n in "$@"; do
    PSGLA_LIB=exp_libs/lib_$n.so timeout -k 10 120 python bench.py --no-cpu --steps 400 --warmup 40 $args > gpurun_out/ab_$n.json
    python - "$n" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:>12s} step {d['ms_per_step']:.4f} ms  kernel {d['roofline']['kernel_ms']:.5f} ms ({d['roofline']['kernel']})  frac {d['roofline']['frac']:.4f}", flush=True)
PY
  done
done
