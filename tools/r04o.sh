#!/bin/bash
# Round 4, call o: issue priority of the row stream's front waves (scheduling only, results bit-identical): product 0,
# fprio1 = 1 (= the stages), fprio2 = 2 (above the stages, below the back), fprioph0 = 2 during the Philox phase only.
set -o pipefail
cd "$(dirname "$0")/.."
tools/ab_bench.sh o64 3 "--steps 400 --warmup 40" prod fprio1 fprio2 fprioph0 || exit 1
tools/ab_bench.sh o481 2 "--steps 100 --warmup 10 --warmup-seconds 0.5 --H 481 --W 321" prod fprio1 fprio2 fprioph0 || exit 1
tools/ab_bench.sh o32 2 "--steps 200 --warmup 20 --warmup-seconds 0.5 --batch 32" prod fprio1 fprio2 fprioph0 || exit 1
