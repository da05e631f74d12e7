set -e
# Host copy rates by L3 placement of the copying threads (tools/host_copy_probe).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06p
mkdir -p $O
cd $R
timeout -k 10 120 $R/tools/host_copy_probe 100 > $O/copy_probe.jsonl 2> $O/copy_probe.err
V="c256_s4:262144:4:0:0,pinned:262144:4:0:0:0:1:ROWS=pinned"
timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep.jsonl 2> $O/sweep.err
