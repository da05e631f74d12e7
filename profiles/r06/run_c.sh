set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r06c
V="c512_s2:524288:2:0:0,c256_s4:262144:4:0:0,c256_s4_f64:262144:4:65536:0,c256_s4_f128:262144:4:131072:0,c256_s3:262144:3:0:0,c384_s3:393216:3:0:0,c192_s4:196608:4:0:0,c512_s2_f128:524288:2:131072:0,c512_s4_f128:524288:4:131072:0,c256_s8:262144:8:0:0,c256_s4_gate:262144:4:0:1"
timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $R/gpurun_out/r06c/sweep.jsonl 2> $R/gpurun_out/r06c/sweep.err
cd /tmp && export TMPDIR=/tmp
HRS_HOST_CHUNK=262144 HRS_HOST_SLOTS=4 timeout -k 10 120 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $R/gpurun_out/r06c/trace_c256 -- $R/tools/host_call_rate 20 > $R/gpurun_out/r06c/trace_c256.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $R/gpurun_out/r06c/trace_c512 -- $R/tools/host_call_rate 20 > $R/gpurun_out/r06c/trace_c512.log 2>&1
