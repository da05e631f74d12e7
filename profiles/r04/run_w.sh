#!/bin/bash
# rocprofv3 passes of the bench without the C-ABI call leg (whose small
# launches of the same kernels polluted run_v's per-kernel averages).
set -e
O=gpurun_out/r04w
mkdir -p $O
bash profiles/run_rocprof.sh $O/prof
