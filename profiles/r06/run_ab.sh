set -e
# Host CRC fold with the rows' chains interleaved: CRC host-path tests, the
# staged call (host fold vs GPU fold), bench's host_calls leg, and a kernel
# trace of the synchronous calls.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ab
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_host_crc.py tests/test_host_path.py tests/test_async.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1
V="default:0:0:0:0:1,gpufold:0:0:0:0:1:0,pinned:0:0:0:0:1:1:ROWS=pinned"
timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep.jsonl 2> $O/sweep.err
timeout -k 10 200 python -c "import bench, json, torch; from lambdafs_amd import HipReedSolomonCode as C; bench.HipReedSolomonCode = C; bench.torch = torch; print(json.dumps(bench.host_calls(0)))" > $O/bench_host_calls.jsonl 2> $O/bench_host_calls.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o host_calls -- $R/tools/host_call_rate 100 > $O/prof.log 2>&1
