#!/bin/bash
# Round 5: the default bench line with the new legs (async_rounds, e2e_device_set).
set -e
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 500 python bench.py > $O/bench.jsonl 2> $O/bench.err
