set -e
# Smaller first chunks on the final defaults (HRS_HOST_FIRST), interleaved.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ac
mkdir -p $O
cd $R
V="default:0:0:0:0:1,f64k:131072:8:65536:0:1,f32k:131072:8:32768:0:1,c160_f64k:163840:8:65536:0:1,pinned:0:0:0:0:1:1:ROWS=pinned"
timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep.jsonl 2> $O/sweep.err
timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep2.jsonl 2> $O/sweep2.err
