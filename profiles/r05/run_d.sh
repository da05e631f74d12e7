#!/bin/bash
# Round 5: where a synchronous encodeBulk / decodeBulk
# call spends its ~0.33 ms. HIP runtime + kernel + memory-copy trace of the
# C-ABI call-rate tool (no counters), and the plain rate beside it.
set -e
O=$(realpath -m gpurun_out/r05d)
REPO=$(pwd)
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/host_call_rate 300 > $O/rate.jsonl 2> $O/rate.err
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- \
  $REPO/tools/host_call_rate 40 > $O/trace_rate.jsonl 2> $O/trace_rate.err
