#!/bin/bash
# Round-3 second GPU pass: -m gpu suite, the bench, then the rocprofv3
# kernel trace and the FETCH / WRITE / SQ counter passes of the same bench
# command (profiles/run_rocprof.sh), each step under its own time limit.
set -e
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 300 python bench.py > $O/bench.jsonl 2> $O/bench.err
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
bash profiles/run_rocprof.sh $O/prof --no-e2e
