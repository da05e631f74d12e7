#!/bin/bash
# Round-3 fourth GPU pass: fused encode + CRC slicing-table replication A/B
# (HRS_CRC_REP = 32 / 16 / 8 / 4), timing interleaved in one process, then one
# SQ counter pass per variant (8 SQ counters each, own process, KILL after 90 s).
set -e
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 240 python tools/bench_crc_rep.py --reps 3 --iters 10 > $O/crc_rep_ab.jsonl 2> $O/crc_rep_ab.err
export TMPDIR=/tmp
REPO=$(pwd)
for R in 32 16 8 4; do
  (cd /tmp && HRS_CRC_REP=$R timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $REPO/$O/pmc_r$R -o run -- python3 $REPO/tools/bench_crc_rep.py --reps 1 --iters 3 --reps-list $R --no-check > $REPO/$O/pmc_r$R.log 2>&1)
done
