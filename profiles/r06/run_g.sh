set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06g
mkdir -p $O
V="c256_s4:262144:4:0:0,q64:65536:1:0:2:0,q128:131072:1:0:2:0,q256:262144:1:0:2:0,q64uc:65536:1:0:2:1,q128uc:131072:1:0:2:1,q256uc:262144:1:0:2:1"
HRS_HOST_PIECE=262144 timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep.jsonl 2> $O/sweep.err
cd /tmp && export TMPDIR=/tmp
HRS_HOST_QUEUE=1 HRS_HOST_QCHUNK=131072 timeout -k 10 120 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/trace_q128 -- $R/tools/host_call_rate 20 > $O/trace_q128.log 2>&1
