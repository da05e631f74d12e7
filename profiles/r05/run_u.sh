#!/bin/bash
# Round 5: concurrent synchronous calls (bench.py sync_threads), direct vs
# staged, 2 passes each, interleaved.
O=gpurun_out/r05u
mkdir -p $O
for rep in 1 2; do
  for d in 1 0; do
    HRS_HOST_DIRECT=$d timeout -k 10 120 python -c "import json, bench, lambdafs_amd; bench.HipReedSolomonCode = lambdafs_amd.HipReedSolomonCode; print(json.dumps(bench.sync_threads(0, codecs=(1, 2, 3, 4), calls=64)))" \
      >> $O/sync_threads_d$d.jsonl 2>> $O/err.txt || exit $?
  done
done
