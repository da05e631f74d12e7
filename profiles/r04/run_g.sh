#!/bin/bash
# Fold tables tracked per stream (no cross-stream waits): host-buffer call
# rates, checksummed ones included, and the CRC / async / host suites.
set -e
O=gpurun_out/r04g2
mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 python tools/bench_host_api.py --calls 40 > $O/host_api_$r.jsonl 2> $O/host_api_$r.err
done
HRS_HOST_THREADS=2 timeout -k 10 120 python tools/bench_host_api.py --calls 40 > $O/host_api_t2.jsonl 2> $O/host_api_t2.err
timeout -k 10 600 python -u -m pytest tests/test_crc32.py tests/test_host_crc.py tests/test_async.py tests/test_jni.py tests/test_cpp_harness.py tests/test_encode_crc.py tests/test_decode_crc.py -m gpu -x -v --timeout 500 --timeout-method thread > $O/gpu_tests_crc.txt 2>&1
