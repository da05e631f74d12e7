set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06e
mkdir -p $O
timeout -k 10 120 $R/tools/host_copy_probe 200 > $O/copy_probe.jsonl 2>&1
V="c256_s4:262144:4:0:0:0,c256_s4_nt:262144:4:0:0:1,c512_s2:524288:2:0:0:0,c512_s2_nt:524288:2:0:0:1,c256_s8_nt:262144:8:0:0:1,c128_s4_nt:131072:4:0:0:1"
HRS_HOST_PIECE=262144 timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep.jsonl 2> $O/sweep.err
