set -e
# Final-code rocprofv3 evidence for the bench workload: kernel trace + FETCH /
# WRITE / SQ passes (profiles/run_rocprof.sh), each pass its own run.
R=$GRAFT_REPO_ROOT
cd $R
bash profiles/run_rocprof.sh gpurun_out/r06an/prof
