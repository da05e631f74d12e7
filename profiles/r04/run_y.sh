#!/bin/bash
# Time-phased writes with the period set from the previous launch's measured
# read-phase task time (tools/gather_lab.hip calib mode).
set -e
O=gpurun_out/r04y
mkdir -p $O
timeout -k 10 200 ./tools/gather_lab 12 calib > $O/calib.jsonl 2> $O/calib.err
timeout -k 10 120 ./tools/gather_lab 7 > $O/gather_lab.jsonl 2> $O/gather_lab.err
