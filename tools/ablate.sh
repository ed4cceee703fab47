#!/bin/bash
# One GPU call: bench.py kernel timing for every diagnostic build in exp_libs/ (see build_variants.sh).
# Usage: tools/ablate.sh OUT "name[:extra bench args]" ...
out=$1; shift
mkdir -p gpurun_out
: > gpurun_out/$out
for spec in "$@"; do
  name=${spec%%:*}; extra=""
  [ "$name" != "$spec" ] && extra=${spec#*:}
  PSGLA_LIB=$PWD/exp_libs/lib_$name.so timeout -k 10 120 python bench.py --no-cpu --steps 200 --warmup 20 $extra > gpurun_out/_b.json 2> gpurun_out/_b.err || { echo "FAIL $spec" >> gpurun_out/$out; tail -5 gpurun_out/_b.err >> gpurun_out/$out; exit 1; }
  python - "$spec" >> gpurun_out/$out <<'PY'
import json, sys
d = json.load(open("gpurun_out/_b.json"))
print(f"{sys.argv[1]:40s} step_ms={d['ms_per_step']:.4f} kernel_ms={d['roofline']['kernel_ms']:.4f} frac={d['roofline']['frac']:.3f}")
PY
done
cat gpurun_out/$out
