#!/bin/bash
# Validation of the tree after the checksummed zero copy and the bench's
# host_calls leg: C-ABI call rates by chunk x transfer mode, the full GPU
# suite, smoke, the default bench.
set -e
O=gpurun_out/r04n
mkdir -p $O
for ch in 262144 524288 1048576; do
  for zc in 1 0; do
    HRS_HOST_CHUNK=$ch HRS_ZEROCOPY=$zc timeout -k 10 120 ./tools/host_call_rate 300 > $O/rate_c${ch}_zc$zc.jsonl 2> $O/rate_c${ch}_zc$zc.err
  done
done
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 400 python bench.py > $O/bench.jsonl 2> $O/bench.err
