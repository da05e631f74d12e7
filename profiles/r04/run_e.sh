#!/bin/bash
# Round 4, fifth pass: zero-copy defaults (grid cap 64, copy threads from the
# CPU share): the sync-call sweep by threads x chunk, the host-batch A/B with
# caps below 64 and with 8 copy threads.
set -e
O=gpurun_out/r04e
mkdir -p $O
for t in 2 4 8 16; do
  for ch in 262144 524288 1048576; do
    HRS_HOST_THREADS=$t HRS_HOST_CHUNK=$ch timeout -k 10 120 python tools/bench_host_ab.py --calls 30 > $O/host_ab_t${t}_c$ch.jsonl 2> $O/host_ab_t${t}_c$ch.err
  done
done
timeout -k 10 120 python tools/bench_host_ab.py --calls 30 > $O/host_ab_default.jsonl 2> $O/host_ab_default.err
timeout -k 10 300 python tools/bench_hbatch.py --reps 4 > $O/hbatch_ab.jsonl 2> $O/hbatch_ab.err
HRS_HOST_THREADS=2 timeout -k 10 300 python tools/bench_hbatch.py --reps 3 --zc-blocks > $O/hbatch_ab_t2.jsonl 2> $O/hbatch_ab_t2.err
