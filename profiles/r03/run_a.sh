#!/bin/bash
# Round-3 first GPU pass: the full -m gpu suite, the bench, the layout probe
# and the decode-kernel A/B. Each step has its own time limit; any failure ends the script.
set -e
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 300 python bench.py > $O/bench.jsonl 2> $O/bench.err
timeout -k 10 180 ./tools/layout_probe 7 > $O/layout_probe.txt 2>&1
timeout -k 10 180 python tools/bench_decode_ab.py > $O/decode_ab.jsonl 2>&1
