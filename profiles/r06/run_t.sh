set -e
# Same box: bench.py's host_calls leg (Python / ctypes, numpy rows) against
# the C sweep and host_call_rate on the same calls.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06t
mkdir -p $O
cd $R
timeout -k 10 200 python -c "import bench, json; print(json.dumps(bench.host_calls(0))); print(json.dumps(bench.host_calls(0)))" > $O/bench_host_calls.jsonl 2> $O/bench_host_calls.err
V="default:0:0:0:0,c256_s4:262144:4:0:0,pinned:262144:4:0:0:0:1:ROWS=pinned"
timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep.jsonl 2> $O/sweep.err
timeout -k 10 100 $R/tools/host_call_rate 100 > $O/host_call_rate.jsonl 2> $O/host_call_rate.err
timeout -k 10 200 python -c "import bench, json; print(json.dumps(bench.host_calls(0)))" >> $O/bench_host_calls.jsonl 2>> $O/bench_host_calls.err
