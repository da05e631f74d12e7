#!/bin/bash
# Block-range task order: edge-shape parity under both orders, the order A/B
# over every streaming kernel, the full GPU suite, then the default bench.
set -e
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_task_order.py -x -q --timeout 240 --timeout-method thread > $O/order_tests.txt 2>&1
timeout -k 10 400 python -u tools/bench_order.py --iters 10 --reps 3 > $O/order_ab.jsonl 2> $O/order_ab.err
timeout -k 10 300 ./tools/sched_lab 7 > $O/sched_lab.jsonl 2> $O/sched_lab.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 400 python bench.py > $O/bench.jsonl 2> $O/bench.err
