#!/bin/bash
# Synchronous call rate through the C ABI (the JNI shim's calls, no Python
# marshalling): chunk sizes x transfer mode.
set -e
O=gpurun_out/r04m
mkdir -p $O
for ch in 262144 524288 1048576; do
  for zc in 1 0; do
    HRS_HOST_CHUNK=$ch HRS_ZEROCOPY=$zc timeout -k 10 120 ./tools/host_call_rate 300 > $O/rate_c${ch}_zc$zc.jsonl 2> $O/rate_c${ch}_zc$zc.err
  done
done
