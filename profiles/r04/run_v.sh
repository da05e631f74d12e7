#!/bin/bash
# Round 4 final pass on the final kernels (window-order argument, grid-stride
# default): the full GPU suite, smoke, the default bench, the C-ABI call
# rates, then the rocprofv3 kernel trace and the FETCH / WRITE / SQ counter
# passes of the bench (profiles/run_rocprof.sh).
set -e
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 400 python bench.py > $O/bench.jsonl 2> $O/bench.err
timeout -k 10 120 ./tools/host_call_rate 300 > $O/host_call_rate.jsonl 2> $O/host_call_rate.err
bash profiles/run_rocprof.sh $O/prof
