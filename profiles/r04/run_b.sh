#!/bin/bash
# Round 4, second GPU pass: the probe-library split, combinable digests,
# the 8-rank real-bench test, duplex host batches (A/B), copy lab rerun.
set -e
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 240 ./tools/copy_lab 7 4 > $O/copy_lab.jsonl 2> $O/copy_lab.err
timeout -k 10 120 ./tools/memcpy_probe 60 > $O/memcpy_probe.jsonl 2> $O/memcpy_probe.err
timeout -k 10 300 python tools/bench_hbatch.py --reps 5 > $O/hbatch_ab.jsonl 2> $O/hbatch_ab.err
timeout -k 10 900 python -u -m pytest tests/test_probes.py tests/test_host_batch.py tests/test_rs_legacy.py tests/test_crc32.py tests/test_jni.py tests/test_async.py tests/test_gpu_full_digests.py tests/test_multirank_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests_sel.txt 2>&1
timeout -k 10 300 python tools/bench_decode_crc.py --reps 5 --erased "4;0,5;2,9;1,6,11" > $O/dcrc_ab.jsonl 2> $O/dcrc_ab.err
timeout -k 10 400 python bench.py > $O/bench.jsonl 2> $O/bench.err
