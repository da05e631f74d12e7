#!/bin/bash
# The copy pool's own rate on the box, by worker count.
set -e
O=gpurun_out/r04i
mkdir -p $O
for t in 0 1 2 4 8 15; do
  HRS_HOST_THREADS=$t timeout -k 10 60 ./tools/pool_probe > $O/pool_t$t.jsonl 2> $O/pool_t$t.err
done
timeout -k 10 60 ./tools/memcpy_probe 60 > $O/memcpy_probe.jsonl 2> $O/memcpy_probe.err
