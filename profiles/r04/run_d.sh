#!/bin/bash
# Round 4, fourth pass: zero-copy host paths — A/B against the copy-engine
# pipelines, grid caps, sync calls by chunk size; then the host-path tests.
set -e
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 300 python tools/bench_hbatch.py --reps 4 > $O/hbatch_ab.jsonl 2> $O/hbatch_ab.err
for ch in 262144 524288 1048576; do
  HRS_HOST_CHUNK=$ch timeout -k 10 120 python tools/bench_host_ab.py --calls 30 > $O/host_ab_c$ch.jsonl 2> $O/host_ab_c$ch.err
done
HRS_HOST_THREADS=8 timeout -k 10 120 python tools/bench_host_ab.py --calls 30 > $O/host_ab_t8.jsonl 2> $O/host_ab_t8.err
timeout -k 10 900 python -u -m pytest tests/test_host_batch.py tests/test_host_path.py tests/test_async.py tests/test_jni.py tests/test_cpp_harness.py tests/test_host_crc.py -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests_host.txt 2>&1
