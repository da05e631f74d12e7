#!/bin/bash
# Task-order x block-shape lab for the headline encode (tools/sched_lab.hip).
set -e
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 300 ./tools/sched_lab 9 > $O/sched_lab.jsonl 2> $O/sched_lab.err
