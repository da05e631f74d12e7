#!/bin/bash
# Round-3 third GPU pass: the -m gpu suite and smoke on the current tree, then
# a resident-blocks-per-CU sweep of the RS(10,4) encode and repairs
# (HRS_BLOCKS_PER_CU overrides every streaming kernel's default; one process per setting, 2 reps).
set -e
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
for rep in 1 2; do
  for b in 1 2 3 4; do
    HRS_BLOCKS_PER_CU=$b timeout -k 10 180 python tools/bench_codes.py --codes rs --iters 20 >> $O/bpc_sweep.jsonl 2>> $O/bpc_sweep.err
  done
  timeout -k 10 180 python tools/bench_codes.py --codes rs --iters 20 >> $O/bpc_sweep.jsonl 2>> $O/bpc_sweep.err
done
