set -e
# Staged-call defaults re-checked with nontemporal copy-ins: chunk / slot
# variants interleaved, and 2 / 3 / 4 copy workers (one process each).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06am
mkdir -p $O
cd $R
V="c128_s8:131072:8:0:0:1,c256_s4:262144:4:0:0:1,c192_s6:196608:6:0:0:1,c96_s8:98304:8:0:0:1,c128_s6:131072:6:0:0:1,pinned:0:0:0:0:1:1:ROWS=pinned"
for t in 3 2 4; do
  HRS_HOST_THREADS=$t timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep_t$t.jsonl 2> $O/sweep_t$t.err
done
