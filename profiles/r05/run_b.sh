#!/bin/bash
# Round 5: where the fused encode + CRC kernel's issue
# stalls come from. Three SQ counter passes (each its own run, 8 SQ-block
# counters at most; the SQC_* instruction-cache counters count in the SQ
# block) over tools/bench_encode_crc.py, which launches the fused kernel, the
# plain encode and the CRC pass of the same 1,024 x 1 MiB RS(10,4) batch.
set -e
O=$(realpath -m gpurun_out/r05b)
REPO=$(pwd)
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU2"
P3="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_WAIT_ANY SQ_BUSY_CYCLES"
i=1
for P in "$P1" "$P2" "$P3"; do
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/pmc$i -o run -- \
    python3 $REPO/tools/bench_encode_crc.py --iters 2 > $O/pmc$i.log 2>&1
  i=$((i+1))
done
