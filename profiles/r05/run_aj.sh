#!/bin/bash
# Round 5: small device batches — kernel-trace durations
# next to the HIP-event times of tools/order_shapes.py (default order only).
O=gpurun_out/r05aj
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 tools/order_shapes.py --orders 1 --iters 8 --reps 2 > $O/order_shapes.jsonl 2> $O/err.txt
