#!/bin/bash
# Round 4, call t: issue priorities of the row stream's stage / back waves (scheduling only, bit-identical results):
# product = stages 1, back 3; sprio2 = stages 2; sprlate = stages 6-10 at 2; bprio2 = back 2.
set -o pipefail
cd "$(dirname "$0")/.."
tools/ab_bench.sh t64 3 "--steps 400 --warmup 40" prod sprio2 sprlate bprio2 || exit 1
tools/ab_bench.sh t481 2 "--steps 100 --warmup 10 --warmup-seconds 0.5 --H 481 --W 321" prod sprio2 sprlate bprio2 || exit 1
