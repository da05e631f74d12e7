#!/bin/bash
# Round 5 A/B: concurrent synchronous callers with direct calls allowed to
# overlap (default) vs one direct call at a time (HRS_HOST_DIRECT_EXCL=1, the
# others staged), vs all staged. 3 passes, interleaved.
O=gpurun_out/r05z
mkdir -p $O
for rep in 1 2 3; do
  for mode in shared excl staged; do
    case $mode in
      shared) env_="HRS_HOST_DIRECT=1 HRS_HOST_DIRECT_EXCL=0" ;;
      excl) env_="HRS_HOST_DIRECT=1 HRS_HOST_DIRECT_EXCL=1" ;;
      staged) env_="HRS_HOST_DIRECT=0" ;;
    esac
    env $env_ timeout -k 10 120 python -c "import json, bench, lambdafs_amd; bench.HipReedSolomonCode = lambdafs_amd.HipReedSolomonCode; print(json.dumps(bench.sync_threads(0, codecs=(1, 2, 4), calls=96)))" \
      >> $O/$mode.jsonl 2>> $O/err.txt || exit $?
  done
done
