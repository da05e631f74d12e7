#!/bin/bash
# Round-3 validation of the final tree: GPU suite, smoke, default bench,
# then the synchronous host-buffer calls (decodeBulkCrc now fused per chunk).
set -e
O=gpurun_out/r03v9
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 400 python bench.py > $O/bench.jsonl 2> $O/bench.err
timeout -k 10 300 python tools/bench_host_api.py > $O/host_api.jsonl 2> $O/host_api.err
