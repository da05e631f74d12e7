set -e
# Same box: bench.py's host_calls leg against the C sweep and per-call
# distributions from Python (tools/host_call_stats.py) under pool variants.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06v
mkdir -p $O
cd $R
timeout -k 10 200 python -c "import bench, json, torch; from lambdafs_amd import HipReedSolomonCode as C; bench.HipReedSolomonCode = C; bench.torch = torch; print(json.dumps(bench.host_calls(0))); print(json.dumps(bench.host_calls(0)))" > $O/bench_host_calls.jsonl 2> $O/bench_host_calls.err
timeout -k 10 100 python tools/host_call_stats.py 300 default >> $O/stats.jsonl 2>> $O/stats.err
HRS_HOST_PIN=0 timeout -k 10 100 python tools/host_call_stats.py 300 pin0 >> $O/stats.jsonl 2>> $O/stats.err
HRS_HOST_THREADS=2 timeout -k 10 100 python tools/host_call_stats.py 300 t2 >> $O/stats.jsonl 2>> $O/stats.err
HRS_HOST_CHUNK=262144 HRS_HOST_SLOTS=4 timeout -k 10 100 python tools/host_call_stats.py 300 c256s4 >> $O/stats.jsonl 2>> $O/stats.err
V="default:0:0:0:0,c256_s4:262144:4:0:0"
timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep.jsonl 2> $O/sweep.err
timeout -k 10 100 $R/tools/host_call_rate 100 > $O/host_call_rate.jsonl 2> $O/host_call_rate.err
nproc > $O/cpus.txt; taskset -p $$ >> $O/cpus.txt; lscpu | grep -i "L3\|NUMA" >> $O/cpus.txt
timeout -k 10 400 python bench.py > $O/bench.jsonl 2> $O/bench.err
