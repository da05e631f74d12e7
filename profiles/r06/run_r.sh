set -e
# Chunk / slot sizes with the reworked copy pool, and piece size / workers
# (process-level knobs, one process each).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06r
mkdir -p $O
cd $R
V="c128_s8:131072:8:0:0,pinned:262144:4:0:0:0:1:ROWS=pinned,c64_s8:65536:8:0:0,c128_s6:131072:6:0:0,c192_s6:196608:6:0:0,c256_s4:262144:4:0:0,c96_s8:98304:8:0:0"
for cfg in "2 262144" "3 262144" "3 65536" "2 65536"; do
  set -- $cfg
  HRS_HOST_THREADS=$1 HRS_HOST_PIECE=$2 timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep_t$1_p$2.jsonl 2> $O/sweep_t$1_p$2.err
done
