#!/bin/bash
# wave-kernel bring-up: parity tests, then the default bench with the stream and wave kernels side by side
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "wave" > gpurun_out/wave_tests.log 2>&1
rc=$?
tail -15 gpurun_out/wave_tests.log
[ $rc -eq 0 ] || exit $rc
for v in stream wave stream wave; do
  timeout -k 10 200 python3 bench.py --no-cpu --variant $v >> gpurun_out/wave_bench.jsonl 2>> gpurun_out/wave_bench.err || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/wave_bench.jsonl'):
    d=json.loads(l); r=d['roofline']; print(r['kernel'], d['ms_per_step'], r['kernel_ms'], r['frac'])"
