#!/bin/bash
# Interleaved A/B of libraries within ONE GPU call: for each repetition, every library in turn runs bench.py
# with the same arguments (no CPU leg).  "prod" = the product library; NAME = exp_libs/lib_NAME.so; VAR=VALUE = the
# product library with that environment variable set (e.g. PSGLA_STREAM_LAYOUT=2); prodN@ARGS = the product library
# with extra bench arguments ARGS (a leg named prodN).
# stdout/stderr of every leg are kept (gpurun_out/ab_TAG/<lib>_<rep>.{json,err}); a failing leg ends the script
# with its stderr printed.  One line per leg: tag | lib | rep | ms_per_step | kernel_ms | kernel.
# Usage: tools/ab_bench.sh TAG REPS "BENCH ARGS" lib1 lib2 ...
set -o pipefail
cd "$(dirname "$0")/.."
T=$1; REPS=$2; ARGS=$3; shift 3
O=gpurun_out/ab_$T
mkdir -p $O
for rep in $(seq 1 $REPS); do
  for leg in "$@"; do
    # NAME@EXTRA: the leg NAME (prod / lib / VAR=VALUE as above) with EXTRA bench arguments (e.g. prod10@--tile-multi-steps 10:
    # a leg of its own named prod10, run on the product library)
    v=${leg%%@*}; EXTRA=""; [[ "$leg" == *@* ]] && EXTRA=${leg#*@}
    base=${v%%[0-9]*}; [ -n "$EXTRA" ] && [ "$base" = "prod" ] && LV=prod || LV=$v
    if [ "$LV" = "prod" ]; then LIBENV=""; elif [[ "$LV" == *=* ]]; then LIBENV="$LV"; else LIBENV="PSGLA_LIB=exp_libs/lib_$LV.so"; fi
    env $LIBENV timeout -k 10 180 python3 bench.py --no-cpu $ARGS $EXTRA > $O/${v}_$rep.json 2> $O/${v}_$rep.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "leg $v rep $rep failed rc=$rc"; tail -20 $O/${v}_$rep.err; exit $rc; fi
    python3 - "$T" "$v" "$rep" "$O/${v}_$rep.json" <<'PY'
import json, sys
t, v, rep, path = sys.argv[1:]
d = json.loads(open(path).read().strip().splitlines()[-1])
print(f"{t} | {v:>22s} | {rep} | {d['ms_per_step']:.5f} | {d['roofline']['kernel_ms']:.5f} | {d['roofline']['kernel']}", flush=True)
PY
  done
done
