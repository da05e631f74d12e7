#!/bin/bash
# Round 5 rocprofv3 evidence for the bench workload (kernel trace + FETCH /
# WRITE / SQ passes, profiles/run_rocprof.sh) into gpurun_out/r05l/prof.
bash profiles/run_rocprof.sh gpurun_out/r05l/prof
