#!/bin/bash
# Closing profile of a round at a commit, in ONE GPU call: the full GPU suite, stream (64 chains) / tile (8 chains)
# kernel-trace + PMC profiles (tools/profile_round.sh), the one-GPU strong sweep with the driver's command, the
# default bench line (its roofline.traffic from this call's PMC summary), castle timing in both orientations at
# batch 1 and 64, the tile kernel's per-phase budget (only when a phase-stamp build exp_libs/lib_tdiag.so exists:
# tools/variant_build.py tdiag tools/patches/tile_phasediag.py) and the three DNN configurations.
# Usage: tools/close_round.sh TAG COMMIT [--no-tests] [--no-dnn]
set -o pipefail
cd "$(dirname "$0")/.."
T=${1:?tag}; C=${2:-unknown}; shift 2
TESTS=1; DNN=1
for a in "$@"; do
  case $a in --no-tests) TESTS=0 ;; --no-dnn) DNN=0 ;; esac
done
mkdir -p gpurun_out
if [ $TESTS = 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 \
    || { tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
  tail -1 gpurun_out/${T}_gpu_tests.log
fi
tools/profile_round.sh ${T}64 $C tv_stream_kernel 64 > gpurun_out/${T}_prof64.log 2>&1 || { tail -20 gpurun_out/${T}_prof64.log; exit 1; }
tools/profile_round.sh ${T}8 $C tv_tile_kernel 8 > gpurun_out/${T}_prof8.log 2>&1 || { tail -20 gpurun_out/${T}_prof8.log; exit 1; }
tools/bench_sweep.sh gpurun_out/${T}_sweep.jsonl > /dev/null || exit 1
python3 -c "
import json
for l in open('gpurun_out/${T}_sweep.jsonl'):
    d = json.loads(l); print(d['config']['chains_per_gpu'], d['roofline']['kernel'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python3 bench.py --pmc-json gpurun_out/prof_${T}64/pmc.json > gpurun_out/${T}_bench.json || exit 1
tail -c 900 gpurun_out/${T}_bench.json
: > gpurun_out/${T}_castle.jsonl
for args in "10000 1" "10000 1 T" "2000 64" "2000 64 T"; do
  timeout -k 10 300 python3 tools/castle_timing.py $args >> gpurun_out/${T}_castle.jsonl || exit 1
done
cat gpurun_out/${T}_castle.jsonl
if [ -f exp_libs/lib_tdiag.so ]; then
  : > gpurun_out/${T}_tile_phases.txt
  for shape in "8 256 256" "1 481 321" "1 321 481"; do
    PSGLA_LIB=exp_libs/lib_tdiag.so timeout -k 10 120 python3 tools/tile_phasediag.py $shape >> gpurun_out/${T}_tile_phases.txt 2>&1 \
      || { tail -20 gpurun_out/${T}_tile_phases.txt; exit 1; }
  done
  grep -v "amdgpu.ids" gpurun_out/${T}_tile_phases.txt
fi
if [ $DNN = 1 ]; then
  : > gpurun_out/${T}_dnn.jsonl
  for w in dncnn-inpaint dncnn-deblur drunet-ula; do
    timeout -k 10 300 python3 tools/bench_dnn.py --workload $w --channels-last >> gpurun_out/${T}_dnn.jsonl || exit 1
  done
  cat gpurun_out/${T}_dnn.jsonl
fi
