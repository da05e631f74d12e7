#!/bin/bash
# Round 5: zero-copy grid cap sweep for the synchronous calls (one stripe per
# call): host_call_rate (all four call kinds, T = 1) and sync_threads (T = 1, 4).
O=gpurun_out/r05w
mkdir -p $O
for rep in 1 2; do
  for zc in 4 8 12 16 24 32 64; do
    HRS_ZC_BLOCKS=$zc timeout -k 10 60 ./tools/host_call_rate 300 >> $O/rate_zc$zc.jsonl 2>> $O/err.txt || exit $?
    HRS_ZC_BLOCKS=$zc timeout -k 10 120 python -c "import json, bench, lambdafs_amd; bench.HipReedSolomonCode = lambdafs_amd.HipReedSolomonCode; print(json.dumps(bench.sync_threads(0, codecs=(1, 4), calls=64)))" \
      >> $O/threads_zc$zc.jsonl 2>> $O/err.txt || exit $?
  done
done
