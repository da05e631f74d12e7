#!/bin/bash
# Round-3 validation pass of the tree: the -m gpu suite (incl. the single-rank
# RCCL collectives test), smoke, and the default bench.
set -e
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 300 python bench.py > $O/bench.jsonl 2> $O/bench.err
