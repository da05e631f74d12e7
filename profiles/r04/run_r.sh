#!/bin/bash
# Window order by job shape (tools/order_shapes.py).
set -e
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 600 python -u tools/order_shapes.py --iters 8 --reps 3 > $O/order_shapes.jsonl 2> $O/order_shapes.err
