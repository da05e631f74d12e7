#!/bin/bash
# Synchronous C-ABI calls: quarter-size first chunk (HRS_HOST_RAMP=1) vs not,
# interleaved; then the host-path suites with the ramp on.
set -e
O=gpurun_out/r04ramp
mkdir -p $O
for rep in 1 2 3; do
  for ch in 524288 1048576; do
    for r in 0 1; do
      HRS_HOST_CHUNK=$ch HRS_HOST_RAMP=$r timeout -k 10 120 ./tools/host_call_rate 300 > $O/rate_c${ch}_r${r}_$rep.jsonl 2> $O/rate_c${ch}_r${r}_$rep.err
    done
  done
done
HRS_HOST_RAMP=1 timeout -k 10 300 python -u -m pytest tests/test_host_path.py tests/test_host_crc.py tests/test_host_batch.py -x -q --timeout 240 --timeout-method thread > $O/host_tests_ramp.txt 2>&1
