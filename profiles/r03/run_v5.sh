#!/bin/bash
# Round-3: fused repair + CRC with the CRC tail after the next task's loads:
# its suite (DPP lane tree, and the ds_bpermute tree), then fused vs plain
# repair vs two passes (RS(10,4), 1 MiB x 1,024), tree variants alternating.
set -e
O=gpurun_out/r03v5
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_decode_crc.py tests/test_host_crc.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/decode_crc_tests.txt 2>&1
HRS_DCRC_TREE=0 timeout -k 10 300 python -u -m pytest tests/test_decode_crc.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/decode_crc_tests_tree0.txt 2>&1
for rep in 1 2 3; do
  for v in 1 0; do
    HRS_DCRC_TREE=$v timeout -k 10 200 python tools/bench_decode_crc.py --reps 1 | sed "s/^{/{\"dpp_tree\": $v, /" >> $O/decode_crc_ab.jsonl
  done
done
