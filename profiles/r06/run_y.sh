set -e
# Copy-in store default "auto" (nontemporal off the GPU's NUMA node) and the
# pool's workers on the GPU's node: host-path suites, then the staged call by
# store mode unbound and from the other socket, then bench's host_calls leg.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06y
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_host_path.py tests/test_host_batch.py tests/test_host_memory.py tests/test_host_crc.py tests/test_async.py tests/test_async_threads.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1
timeout -k 10 120 $R/tools/host_copy_probe 20 > $O/copy_probe.jsonl 2> $O/copy_probe.err
GN=$(python3 -c "import json; print(json.loads(open('$O/copy_probe.jsonl').readline())['gpu_node'])")
if [ "$GN" -lt 0 ]; then GN=0; fi
ON=$((1 - GN))
GC=$(cat /sys/devices/system/node/node$GN/cpulist)
OC=$(cat /sys/devices/system/node/node$ON/cpulist)
echo "gpu_node=$GN gpu_cpus=$GC other_cpus=$OC" > $O/placement.txt
V="auto:0:0:0:0:auto,plain:0:0:0:0:0,nt:0:0:0:0:1,pinned:0:0:0:0:auto:1:ROWS=pinned"
S="$R/tools/host_pipeline_sweep 100 5 1048576 $V"
timeout -k 10 200 $S > $O/unbound.jsonl 2> $O/unbound.err
timeout -k 10 200 taskset -c $OC $S > $O/other.jsonl 2> $O/other.err
timeout -k 10 200 taskset -c $GC $S > $O/gpunode.jsonl 2> $O/gpunode.err
timeout -k 10 200 python -c "import bench, json, torch; from lambdafs_amd import HipReedSolomonCode as C; bench.HipReedSolomonCode = C; bench.torch = torch; print(json.dumps(bench.host_calls(0))); print(json.dumps(bench.sync_threads(0)))" > $O/bench_host_calls.jsonl 2> $O/bench_host_calls.err
