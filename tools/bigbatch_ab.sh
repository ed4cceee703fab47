set -o pipefail
for v in stream wave stream wave; do
  timeout -k 10 200 python3 bench.py --no-cpu --batch 704 --steps 40 --warmup 10 --variant $v > gpurun_out/bigb_$v.json || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/bigb_$v.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$v', d['config']['chains_per_gpu'], r['kernel'], d['ms_per_step'], r['kernel_ms'], r['frac'])"
done
