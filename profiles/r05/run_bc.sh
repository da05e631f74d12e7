#!/bin/bash
# Round 5: the long fuzz sequence three times on the default paths (staged /
# pinned), after the direct path became opt-in.
O=gpurun_out/r05bc
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 400 python -u tests/tools/fuzz_long.py 6 2000 > $O/fuzz_$rep.jsonl 2> $O/fuzz_$rep.err || exit $?
done
