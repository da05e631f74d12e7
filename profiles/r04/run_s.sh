#!/bin/bash
# Rotated block range vs block range vs grid-stride by job shape.
set -e
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_task_order.py -x -q --timeout 240 --timeout-method thread > $O/order_tests.txt 2>&1
timeout -k 10 600 python -u tools/order_shapes.py --iters 8 --reps 3 --orders 1,0,-1  # -1: the dropped scattered-start block range > $O/order_shapes.jsonl 2> $O/order_shapes.err
