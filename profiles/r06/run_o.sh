set -e
# NUMA placement of CPU / rows / staging / GPU; the staged call against the
# in-place floor (ROWS=pinned) and slot counts, with the box's 4 hardware
# queues per process and with 8.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06o
mkdir -p $O
cd $R
timeout -k 10 120 $R/tools/host_copy_probe 100 > $O/copy_probe.jsonl 2> $O/copy_probe.err
V="c256_s4:262144:4:0:0,pinned:262144:4:0:0:0:1:ROWS=pinned,c256_s3:262144:3:0:0,c256_s6:262144:6:0:0,c128_s8:131072:8:0:0"
timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep_q4.jsonl 2> $O/sweep_q4.err
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep_q8.jsonl 2> $O/sweep_q8.err
