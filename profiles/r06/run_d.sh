set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06d
mkdir -p $O
V="c512_s2:524288:2:0:0,c256_s4:262144:4:0:0,c128_s4:131072:4:0:0,c128_s8:131072:8:0:0,c256_s8:262144:8:0:0,c512_s4:524288:4:0:0,c256_s4_gate:262144:4:0:1,c128_s8_gate:131072:8:0:1"
HRS_HOST_PIECE=65536 timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep_p64.jsonl 2> $O/sweep_p64.err
HRS_HOST_PIECE=262144 timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep_p256.jsonl 2> $O/sweep_p256.err
HRS_HOST_PIECE=32768 timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep_p32.jsonl 2> $O/sweep_p32.err
cd /tmp && export TMPDIR=/tmp
HRS_HOST_CHUNK=262144 HRS_HOST_SLOTS=4 timeout -k 10 120 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/trace_c256 -- $R/tools/host_call_rate 20 > $O/trace_c256.log 2>&1
