#!/bin/bash
# PMC passes of the wave kernel (the round profile's four passes + instruction-cache counters)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tools/profile_round.sh r02w ${1:-wip} tv_wave_kernel 64 --variant wave > gpurun_out/profw.log 2>&1 || { tail -20 gpurun_out/profw.log; exit 1; }
O=gpurun_out/prof_r02w
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_SMEM SQ_WAIT_INST_LDS --output-format csv -d $O/pmc5 -o p -- \
  python3 bench.py --steps 40 --warmup 4 --warmup-seconds 0.3 --no-cpu --kernel-iters 5 --batch 64 --variant wave > $O/bench_pmc5.json 2> $O/pmc5.err || echo "pmc5 failed"
python3 - <<'PY'
import json, csv, collections
d = json.load(open('gpurun_out/prof_r02w/pmc.json'))
c = d['counters_per_dispatch']
for k in sorted(c): print(k, round(c[k]))
print(d.get('wave_cycle_split'))
try:
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open('gpurun_out/prof_r02w/pmc5/p_counter_collection.csv')):
        if 'tv_wave_kernel' in r['Kernel_Name']:
            agg[r['Counter_Name']] += float(r['Counter_Value'])
            n[(r['Counter_Name'], r['Dispatch_Id'])] += 1
    disp = len({k[1] for k in n})
    for k, v in agg.items(): print('pmc5', k, round(v / max(disp, 1)))
except Exception as e:
    print('pmc5', e)
PY
grep -h "tv_wave_kernel\|tv_stream" gpurun_out/prof_r02w/kt/*kernel_stats.csv | head -3
