set -e
# Final validation after bench reports placement: whole GPU suite, smoke, bench; then a kernel trace
# of the same bench command and a kernel + HIP API trace of the synchronous
# host calls (tools/host_call_rate) on the final staged defaults.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06aq
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 400 python bench.py > $O/bench.jsonl 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --no-cpu-baseline --no-host-calls > $O/trace_bench.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $O/host_calls -o run -- $R/tools/host_call_rate 50 > $O/host_calls.log 2>&1
