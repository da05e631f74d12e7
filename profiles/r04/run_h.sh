#!/bin/bash
# Kernel trace of the synchronous host-buffer calls (zero copy): kernel
# durations and the gaps between them, to see where a 0.37 ms call goes.
set -e
O=gpurun_out/r04h
mkdir -p $O
R=$(pwd)
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/$O/trace -o run -- python3 $R/tools/bench_host_api.py --calls 40 > $R/$O/trace_host_api.log 2>&1)
