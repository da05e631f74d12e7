#!/bin/bash
# Zero copy for the checksummed host-buffer calls (one-pass kernels only):
# host-path suites in both transfer modes, then the call rates.
set -e
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_host_crc.py tests/test_async.py tests/test_host_path.py tests/test_jni.py tests/test_cpp_harness.py tests/test_decode_crc.py tests/test_encode_crc.py -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1
for r in 1 2; do
  timeout -k 10 120 python tools/bench_host_api.py --calls 40 > $O/host_api_$r.jsonl 2> $O/host_api_$r.err
done
HRS_ZEROCOPY=0 timeout -k 10 120 python tools/bench_host_api.py --calls 40 > $O/host_api_ce.jsonl 2> $O/host_api_ce.err
timeout -k 10 120 ./tests/cpp/codec_harness --async=2 10 4 $((16 << 20)) $((1 << 20)) 1 > $O/harness_async.jsonl 2> $O/harness_async.err
HRS_ZEROCOPY=0 timeout -k 10 120 ./tests/cpp/codec_harness --async=2 10 4 $((16 << 20)) $((1 << 20)) 1 > $O/harness_async_ce.jsonl 2> $O/harness_async_ce.err
