#!/bin/bash
# Round 5: synchronous C-ABI call rate vs the chunk ring:
# slots (HRS_HOST_SLOTS 2-4) x chunk bytes (HRS_HOST_CHUNK), two passes each,
# interleaved so box drift hits every variant alike.
set -e
O=gpurun_out/r05f
mkdir -p $O
for rep in 1 2; do
  for sl in 2 3 4; do
    for ch in 131072 262144 524288 1048576; do
      HRS_HOST_SLOTS=$sl HRS_HOST_CHUNK=$ch timeout -k 10 60 ./tools/host_call_rate 300 \
        > $O/rate_s${sl}_c${ch}_r$rep.jsonl 2> $O/rate_s${sl}_c${ch}_r$rep.err
    done
  done
done
