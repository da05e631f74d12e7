#!/bin/bash
# Round-3: 1-output fused repair + CRC with two tasks' CRC tails interleaved
# (HRS_DCRC_PAIR=1) vs one at a time (0): suites under both, then A/B
# alternating (RS(10,4), 1 MiB x 1,024, data shard 0 lost).
set -e
O=gpurun_out/r03v8
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_decode_crc.py tests/test_host_crc.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/decode_crc_tests.txt 2>&1
HRS_DCRC_PAIR=0 timeout -k 10 300 python -u -m pytest tests/test_decode_crc.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/decode_crc_tests_pair0.txt 2>&1
for rep in 1 2 3; do
  for v in 1 0; do
    HRS_DCRC_PAIR=$v timeout -k 10 200 python tools/bench_decode_crc.py --reps 1 --erased "4;2" | sed "s/^{/{\"pair\": $v, /" >> $O/decode_crc_ab.jsonl
  done
done
