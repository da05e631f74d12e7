#!/bin/bash
# Round 5: catch the direct path's rare corruption with the fuzz's failure
# report: the long fuzz sequence up to 4 times (stops at the first failure).
O=gpurun_out/r05au
mkdir -p $O
for rep in 1 2 3 4; do
  timeout -k 10 300 python -u tests/tools/fuzz_long.py 6 2000 > $O/run_$rep.jsonl 2> $O/run_$rep.err || exit 0
done
