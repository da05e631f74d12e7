#!/bin/bash
# Round 6 rocprofv3 evidence for the bench workload (kernel trace + FETCH /
# WRITE / SQ passes, profiles/run_rocprof.sh) into gpurun_out/r06m/prof, and a
# kernel + HIP API trace of the synchronous host calls (tools/host_call_rate).
set -e
R=$GRAFT_REPO_ROOT
cd $R
bash profiles/run_rocprof.sh gpurun_out/r06m/prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $R/gpurun_out/r06m/host_calls -o run -- $R/tools/host_call_rate 50 > $R/gpurun_out/r06m/host_calls.log 2>&1
