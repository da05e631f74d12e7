#!/bin/bash
# Round 5: the staged synchronous call (now the default) over chunk size x
# slot count x copy threads, RS(10,4) 1 MiB cells (tools/host_call_rate).
O=gpurun_out/r05aw
mkdir -p $O
for rep in 1 2; do
  for ch in 131072 262144 524288 1048576; do
    for sl in 2 3 4; do
      HRS_HOST_CHUNK=$ch HRS_HOST_SLOTS=$sl timeout -k 10 60 ./tools/host_call_rate 200 \
        | sed "s/^{/{\"chunk\": $ch, \"slots\": $sl, \"rep\": $rep, /" >> $O/sweep.jsonl || exit $?
    done
  done
done
for th in 2 4 8 12; do
  HRS_HOST_THREADS=$th timeout -k 10 60 ./tools/host_call_rate 200 | sed "s/^{/{\"threads\": $th, /" >> $O/threads.jsonl || exit $?
done
