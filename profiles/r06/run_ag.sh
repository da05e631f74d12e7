set -e
# Dynamic-LDS attribute set once per (kernel, device): CRC suites, the staged
# call sweep, bench's host_calls leg and a HIP API trace of the host calls.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ag
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_host_crc.py tests/test_encode_crc.py tests/test_decode_crc.py tests/test_crc32.py tests/test_device_set.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1
V="default:0:0:0:0:1,pinned:0:0:0:0:1:1:ROWS=pinned"
timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep.jsonl 2> $O/sweep.err
timeout -k 10 200 python -c "import bench, json, torch; from lambdafs_amd import HipReedSolomonCode as C; bench.HipReedSolomonCode = C; bench.torch = torch; print(json.dumps(bench.host_calls(0)))" > $O/bench_host_calls.jsonl 2> $O/bench_host_calls.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $O/host_calls -o run -- $R/tools/host_call_rate 50 > $O/host_calls.log 2>&1
