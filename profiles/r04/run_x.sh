#!/bin/bash
# Gather vs contiguous reads, with and without the written row (tools/gather_lab.hip).
set -e
O=gpurun_out/r04x
mkdir -p $O
timeout -k 10 120 ./tools/gather_lab 9 > $O/gather_lab.jsonl 2> $O/gather_lab.err
