#!/bin/bash
# Round 5: where the direct path's time goes. Kernel trace of the C-ABI call
# loop direct vs staged, then one kernel + HIP API trace of the direct loop.
O=gpurun_out/r05i
mkdir -p $O
export TMPDIR=/tmp
for d in 1 0; do
  HRS_HOST_DIRECT=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_d$d -o run -- \
    ./tools/host_call_rate 100 > $O/kt_d$d.jsonl 2> $O/kt_d$d.err || exit $?
done
HRS_HOST_DIRECT=1 timeout -k 10 120 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/api_d1 -o run -- \
  ./tools/host_call_rate 40 > $O/api_d1.jsonl 2> $O/api_d1.err
