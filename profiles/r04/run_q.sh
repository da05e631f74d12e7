#!/bin/bash
# Window order sweep (block-cyclic chunks / block range) per kernel family,
# edge-shape parity under four orders, the full GPU suite, the bench.
set -e
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_task_order.py -x -q --timeout 240 --timeout-method thread > $O/order_tests.txt 2>&1
timeout -k 10 500 python -u tools/bench_order.py --iters 8 --reps 3 > $O/order_sweep.jsonl 2> $O/order_sweep.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 400 python bench.py > $O/bench.jsonl 2> $O/bench.err
