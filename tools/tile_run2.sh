set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh || exit 1
mkdir -p gpurun_out/tile
: > gpurun_out/tile/sweep2.jsonl
for b in 8 16; do
  for v in stream tile; do
    timeout -k 10 150 python3 bench.py --steps 100 --warmup 10 --no-cpu --batch $b --variant $v >> gpurun_out/tile/sweep2.jsonl || exit 1
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/tile/sweep2.jsonl"):
    d = json.loads(l)
    print(d["config"]["chains_per_gpu"], d["roofline"]["kernel"], d["ms_per_step"], d["roofline"]["kernel_ms_isolated"], d["roofline"]["frac"])
PY
