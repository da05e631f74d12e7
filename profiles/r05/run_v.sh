#!/bin/bash
# Round 5: concurrent direct synchronous calls vs the zero-copy grid cap
# (HRS_ZC_BLOCKS): does a smaller per-kernel grid help when T kernels share
# the host link?
O=gpurun_out/r05v
mkdir -p $O
for rep in 1 2; do
  for zc in 64 32 16; do
    HRS_ZC_BLOCKS=$zc timeout -k 10 120 python -c "import json, bench, lambdafs_amd; bench.HipReedSolomonCode = lambdafs_amd.HipReedSolomonCode; print(json.dumps(bench.sync_threads(0, codecs=(1, 2, 4), calls=64)))" \
      >> $O/zc$zc.jsonl 2>> $O/err.txt || exit $?
  done
done
