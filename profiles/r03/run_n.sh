#!/bin/bash
# Round-3: the probe sweep (hrs_probe_stream / hrs_probe_rows) — its GPU
# tests, then the default bench whose roofline now carries the pattern ceiling.
set -e
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_probes.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/probe_tests.txt 2>&1
timeout -k 10 400 python bench.py > $O/bench.jsonl 2> $O/bench.err
