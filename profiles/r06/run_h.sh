set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06h
mkdir -p $O
V="c256_s4:262144:4:0:0,c512_s2:524288:2:0:0,q128:131072:1:0:2:0,q256:262144:1:0:2:0,q128uc:131072:1:0:2:1"
for t in 0 1 2 4; do
HRS_HOST_THREADS=$t HRS_HOST_PIECE=262144 timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep_t$t.jsonl 2> $O/sweep_t$t.err
done
for t in 0 2; do HRS_HOST_THREADS=$t timeout -k 10 60 $R/tools/host_copy_probe 200 > $O/copy_t$t.jsonl 2>&1; done
