#!/bin/bash
# Round 5 validation: the whole GPU suite, smoke(), the default bench line.
O=gpurun_out/r05final5
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.txt 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench.jsonl 2> $O/bench.err
