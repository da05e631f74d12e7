#!/bin/bash
# Round 5: which mechanism loses the direct path's writes? The long fuzz
# sequence with the direct path on (HRS_HOST_DIRECT=1), by default and with
# numpy's THP advice off, interleaved, 3 runs each on one box. A failing run
# (an assertion, exit status 1) is recorded and the next one starts; any
# other exit status ends the script.
O=gpurun_out/r05be
mkdir -p $O
for rep in 1 2 3; do
  for v in default nothp; do
    arg=""; [ $v = nothp ] && arg="--no-thp"
    HRS_HOST_DIRECT=1 timeout -k 10 300 python -u tests/tools/fuzz_long.py 6 2000 $arg > $O/${v}_$rep.jsonl 2> $O/${v}_$rep.err
    rc=$?
    echo "$v $rep rc=$rc" >> $O/summary.txt
    if [ $rc -gt 1 ]; then exit $rc; fi
  done
done
