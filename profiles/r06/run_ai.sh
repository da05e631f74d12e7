set -e
# Pageable batch drift: NUMA balancing setting, the probe unbound, bound to
# the GPU's socket, and with the pool's workers on the caller's socket.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ai
mkdir -p $O
cd $R
cat /proc/sys/kernel/numa_balancing > $O/numa_balancing.txt 2>&1 || echo unreadable > $O/numa_balancing.txt
timeout -k 10 120 $R/tools/host_copy_probe 5 > $O/copy_probe.jsonl 2> $O/copy_probe.err
GN=$(python3 -c "import json; print(json.loads(open('$O/copy_probe.jsonl').readline())['gpu_node'])")
if [ "$GN" -lt 0 ]; then GN=0; fi
GC=$(cat /sys/devices/system/node/node$GN/cpulist)
timeout -k 10 300 python -u tools/pageable_gap_probe.py > $O/unbound.jsonl 2> $O/unbound.err
timeout -k 10 300 taskset -c $GC python -u tools/pageable_gap_probe.py > $O/gpunode.jsonl 2> $O/gpunode.err
HRS_HOST_HOME=caller timeout -k 10 300 python -u tools/pageable_gap_probe.py > $O/home_caller.jsonl 2> $O/home_caller.err
