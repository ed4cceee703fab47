set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02a
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r02a/b20_1.json &&
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu --warmup-seconds 0 > gpurun_out/r02a/b20_nowarm.json &&
timeout -k 10 120 python3 bench.py --steps 400 --warmup 40 --no-cpu > gpurun_out/r02a/b400.json &&
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu --exact > gpurun_out/r02a/b20_exact.json &&
tools/bench_sweep.sh gpurun_out/r02a/sweep.jsonl &&
tools/profile_round.sh r02a bdfff00 > gpurun_out/r02a/prof.log 2>&1
