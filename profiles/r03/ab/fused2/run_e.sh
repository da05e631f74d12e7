#!/bin/bash
# Round-3 fifth GPU pass: the fused encode + CRC in its two-blocks-per-CU form
# (HRS_FUSED=5: 640-thread blocks x 2 per CU = 5 waves/SIMD, the 68 KiB
# 16-copy LDS image, lane-tree tables from device memory). First its parity
# suites under the variant, then product vs variant timing in alternating
# processes (3 reps each), RS(10,4) / RS(12,4) / RS(6,3).
set -e
O=gpurun_out/r03e
mkdir -p $O
HRS_FUSED=5 timeout -k 10 300 python -u -m pytest tests/test_encode_crc.py tests/test_host_crc.py tests/test_nrs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_fused5.txt 2>&1
for rep in 1 2 3; do
  for v in 3 5; do
    for kp in "10 4" "12 4" "6 3"; do
      set -- $kp
      HRS_FUSED=$v timeout -k 10 120 python tools/bench_encode_crc.py --k $1 --p $2 --iters 10 | sed "s/^{/{\"variant\": $v, /" >> $O/fused2_ab.jsonl
    done
  done
done
