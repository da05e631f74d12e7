set -e
# Copy pool with spinning completion and L3-bound workers: probe, then the
# staged call with binding off / on and 2-4 workers (one process each).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06q
mkdir -p $O
cd $R
timeout -k 10 120 $R/tools/host_copy_probe 100 > $O/copy_probe.jsonl 2> $O/copy_probe.err
V="c256_s4:262144:4:0:0,pinned:262144:4:0:0:0:1:ROWS=pinned,c128_s4:131072:4:0:0,c128_s8:131072:8:0:0"
for cfg in "0 2" "1 2" "1 3" "1 4"; do
  set -- $cfg
  HRS_HOST_PIN=$1 HRS_HOST_THREADS=$2 timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep_pin$1_t$2.jsonl 2> $O/sweep_pin$1_t$2.err
done
