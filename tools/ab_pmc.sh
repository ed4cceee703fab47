#!/bin/bash
# HBM read / write bytes per launch of the dominant kernel for several libraries in ONE GPU call: one
# rocprofv3 pass per counter group (FETCH_SIZE, WRITE_SIZE: MI355X_MICROARCH.md's TCC slot rules), summarised
# by tools/pmc_summary.py.  Usage: tools/ab_pmc.sh TAG KERNEL "BENCH ARGS" lib1 lib2 ...
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
T=$1; K=$2; ARGS=$3; shift 3
O=gpurun_out/pmc_$T
mkdir -p $O
for v in "$@"; do
  if [ "$v" = "prod" ]; then LIBENV=""; else LIBENV="PSGLA_LIB=exp_libs/lib_$v.so"; fi
  i=0
  for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
    i=$((i + 1))
    env $LIBENV timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/${v}_p$i -o p -- \
      python3 bench.py --steps 40 --warmup 4 --warmup-seconds 0.3 --no-cpu $ARGS \
      > $O/${v}_p$i.json 2> $O/${v}_p$i.err || { echo "pmc $v $c failed"; tail -20 $O/${v}_p$i.err; exit 1; }
  done
  python3 tools/pmc_summary.py --round $T --kernel $K --out $O/${v}.json $O/${v}_p1 $O/${v}_p2 $O/${v}_p3 > /dev/null || exit 1
  python3 - "$v" "$O/${v}.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
c = d["counters_per_dispatch"]
w = d.get("wave_cycle_split", {})
print(f"{sys.argv[1]:>10s} read {d['hbm_read_bytes_per_launch']/1e6:8.2f} MB  write {d['hbm_write_bytes_per_launch']/1e6:8.2f} MB"
      f"  wait_any {w.get('SQ_WAIT_ANY', float('nan')):.3f}  valu {w.get('SQ_ACTIVE_INST_VALU', float('nan')):.3f}", flush=True)
PY
done
