#!/bin/bash
# Round-3: fused repair + CRC, software-pipelined for 2-4 outputs too (local
# accumulators: no v_mov_b64 storm) vs the plain 768-thread kernel
# (HRS_DCRC_PLAIN=1): suites under both, then A/B alternating.
set -e
O=gpurun_out/r03v10
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_decode_crc.py tests/test_host_crc.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/decode_crc_tests.txt 2>&1
HRS_DCRC_PLAIN=1 timeout -k 10 300 python -u -m pytest tests/test_decode_crc.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/decode_crc_tests_plain.txt 2>&1
for rep in 1 2 3; do
  for v in 0 1; do
    HRS_DCRC_PLAIN=$v timeout -k 10 200 python tools/bench_decode_crc.py --reps 1 --erased "4;0,5;0,3;1,6,11;0,3,7,12" | sed "s/^{/{\"plain\": $v, /" >> $O/decode_crc_ab.jsonl
  done
done
