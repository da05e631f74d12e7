#!/bin/bash
# Round-3: fused repair + CRC, plain kernel for 2-4 outputs written inline (no v_mov_b64 storm):
# suites at 512 and 768 threads, then fused vs plain repair vs two passes,
# thread variants alternating (RS(10,4), 1 MiB x 1,024).
set -e
O=gpurun_out/r03v7
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_decode_crc.py tests/test_host_crc.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/decode_crc_tests.txt 2>&1
HRS_DCRC_THREADS=768 timeout -k 10 300 python -u -m pytest tests/test_decode_crc.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/decode_crc_tests_768.txt 2>&1
for rep in 1 2 3; do
  for v in 512 768; do
    HRS_DCRC_THREADS=$v timeout -k 10 200 python tools/bench_decode_crc.py --reps 1 --erased "4;0,5;1,6,11;0,3" | sed "s/^{/{\"threads\": $v, /" >> $O/decode_crc_ab.jsonl
  done
done
