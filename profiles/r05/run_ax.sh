#!/bin/bash
# Round 5: timeline of the staged synchronous call (now the default): kernel +
# HIP API trace of tools/host_call_rate.
O=gpurun_out/r05ax
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/api -o run -- \
  ./tools/host_call_rate 40 > $O/rate.jsonl 2> $O/rate.err
