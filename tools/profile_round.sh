#!/bin/bash
# Round profile of the bench command on the GPU box: kernel-trace stats of the driver's bench command
# and the PMC passes (one counter group per run, MI355X_MICROARCH.md's rocprofv3 rules) summarised by
# tools/pmc_summary.py.  Usage: tools/profile_round.sh TAG COMMIT KERNEL CHAINS [extra bench args]
# (writes gpurun_out/prof_TAG*; copy the summaries into profiles/)
set -e
cd "$(dirname "$0")/.."
R=${1:-r02}
COMMIT=${2:-unknown}
KERNEL=${3:-tv_stream_kernel}
CHAINS=${4:-64}
shift 4 || true
EXTRA="--batch $CHAINS $*"
export TMPDIR=/tmp
O=gpurun_out/prof_$R
mkdir -p $O
CMD="bench.py --steps 20 --warmup 5 --no-cpu $EXTRA"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o p -- \
  python3 $CMD > $O/bench_kt.json
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_INSTS_VALU_TRANS_F32"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc$i -o p -- \
    python3 bench.py --steps 40 --warmup 4 --warmup-seconds 0.3 --no-cpu $EXTRA > $O/bench_pmc$i.json
done
python3 tools/pmc_summary.py --round $R --kernel $KERNEL --chains $CHAINS --commit $COMMIT --command "python3 $CMD" \
  --out $O/pmc.json $O/pmc1 $O/pmc2 $O/pmc3 $O/pmc4
