#!/bin/bash
# Copy pool: workers drain whole batches. Pool rate by worker count, the
# synchronous calls and the pageable host batches on this tree.
set -e
O=gpurun_out/r04j
mkdir -p $O
for t in 0 2 4 8 15; do
  HRS_HOST_THREADS=$t timeout -k 10 60 ./tools/pool_probe > $O/pool_t$t.jsonl 2> $O/pool_t$t.err
done
for r in 1 2; do
  timeout -k 10 120 python tools/bench_host_api.py --calls 40 > $O/host_api_$r.jsonl 2> $O/host_api_$r.err
done
timeout -k 10 120 python tools/bench_host_ab.py --calls 40 > $O/host_ab.jsonl 2> $O/host_ab.err
for t in 4 15; do
  HRS_HOST_THREADS=$t timeout -k 10 120 python tools/bench_host_ab.py --calls 40 > $O/host_ab_t$t.jsonl 2> $O/host_ab_t$t.err
done
timeout -k 10 300 python tools/bench_hbatch.py --reps 3 --zc-blocks > $O/hbatch_ab.jsonl 2> $O/hbatch_ab.err
timeout -k 10 120 ./tests/cpp/codec_harness --threads=1 --rounds=64 10 4 > $O/harness_t1.jsonl 2> $O/harness_t1.err
timeout -k 10 120 ./tests/cpp/codec_harness --threads=4 --rounds=32 10 4 > $O/harness_t4.jsonl 2> $O/harness_t4.err
