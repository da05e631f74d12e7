#!/bin/bash
# Round 5, direct path now opt-in: the whole GPU suite, then the long fuzz
# sequence twice on the default (staged) paths.
O=gpurun_out/r05av
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.txt 2>&1 || exit $?
for rep in 1 2; do
  timeout -k 10 400 python -u tests/tools/fuzz_long.py 6 2000 > $O/fuzz_$rep.jsonl 2> $O/fuzz_$rep.err || exit $?
done
