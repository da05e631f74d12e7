#!/bin/bash
# Round 5: interleaved A/B of the staged call layouts, 4 passes.
O=gpurun_out/r05az
mkdir -p $O
for rep in 1 2 3 4; do
  for cfg in "1 524288 2" "0 524288 2" "0 262144 4" "1 262144 4"; do
    set -- $cfg
    HRS_HOST_ONE_STREAM=$1 HRS_HOST_CHUNK=$2 HRS_HOST_SLOTS=$3 timeout -k 10 60 ./tools/host_call_rate 300 \
      | sed "s/^{/{\"one\": $1, \"chunk\": $2, \"slots\": $3, \"rep\": $rep, /" >> $O/ab.jsonl || exit $?
  done
done
