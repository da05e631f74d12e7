#!/bin/bash
# Round 4, third pass: stream structures for a duplex H2D/D2H pipeline.
set -e
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 300 python tools/duplex_pipeline_probe.py --reps 4 > $O/pipeline_probe.jsonl 2> $O/pipeline_probe.err
timeout -k 10 300 python tools/zero_copy_probe.py --reps 5 > $O/zero_copy.jsonl 2> $O/zero_copy.err
