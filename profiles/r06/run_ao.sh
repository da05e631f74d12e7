set -e
# Checksummed staged calls at 128 KiB x 8: narrow fused blocks vs 1,024-thread
# ones, and the zero-copy grid cap, interleaved (two passes).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ao
mkdir -p $O
cd $R
V="default:0:0:0:0:1,wide_blocks:0:0:0:0:1:1:HRS_FUSED_NARROW=0,zc128:0:0:0:0:1:1:HRS_ZC_BLOCKS=128,zc32:0:0:0:0:1:1:HRS_ZC_BLOCKS=32,nocap:0:0:0:0:1:1:HRS_ZC_BLOCKS=0"
timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep1.jsonl 2> $O/sweep1.err
timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep2.jsonl 2> $O/sweep2.err
