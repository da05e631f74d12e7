#!/bin/bash
# Round 5: direct vs staged synchronous calls over the cell size, to place
# HRS_HOST_DIRECT_MIN. RS(10,4) and RS(6,3) (config 2's code), heap rows.
O=gpurun_out/r05o
mkdir -p $O
for kp in "10 4" "6 3"; do
  set -- $kp
  for L in 16384 32768 49152 65536 98304 131072 262144 524288 1048576; do
    for d in 1 0; do
      HRS_HOST_DIRECT=$d HRS_HOST_DIRECT_MIN=0 HRS_HOST_DIRECT_MIN_CRC=0 timeout -k 10 60 ./tools/host_call_rate 300 $L $1 $2 \
        >> $O/sweep_d$d.jsonl 2>> $O/sweep.err || exit $?
    done
  done
done
