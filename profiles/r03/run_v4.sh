#!/bin/bash
# Round-3: the fused repair + CRC suite first, then the re-entry validation
# (GPU suite, smoke, default bench with the decode_crc leg).
set -e
O=gpurun_out/r03v4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_decode_crc.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/decode_crc_tests.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 400 python bench.py > $O/bench.jsonl 2> $O/bench.err
