set -e
# Copy-pool home node (HRS_HOST_HOME: the GPU's NUMA node vs the caller's) and
# copy-in stores (HRS_HOST_NT 0 / 1 / auto) by process placement, one box.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06x
mkdir -p $O
cd $R
timeout -k 10 120 $R/tools/host_copy_probe 20 > $O/copy_probe.jsonl 2> $O/copy_probe.err
GN=$(python3 -c "import json; print(json.loads(open('$O/copy_probe.jsonl').readline())['gpu_node'])")
if [ "$GN" -lt 0 ]; then GN=0; fi
ON=$((1 - GN))
GC=$(cat /sys/devices/system/node/node$GN/cpulist)
OC=$(cat /sys/devices/system/node/node$ON/cpulist)
echo "gpu_node=$GN gpu_cpus=$GC other_cpus=$OC" > $O/placement.txt
V="plain:0:0:0:0:0,nt:0:0:0:0:1,ntauto:0:0:0:0:auto,pinned:0:0:0:0:0:1:ROWS=pinned"
S="$R/tools/host_pipeline_sweep 100 5 1048576 $V"
HRS_HOST_HOME=caller timeout -k 10 200 taskset -c $OC $S > $O/other_caller.jsonl 2> $O/other_caller.err
timeout -k 10 200 taskset -c $OC $S > $O/other_gpu.jsonl 2> $O/other_gpu.err
HRS_HOST_HOME=caller timeout -k 10 200 taskset -c $GC $S > $O/gpunode_caller.jsonl 2> $O/gpunode_caller.err
timeout -k 10 200 taskset -c $GC $S > $O/gpunode_gpu.jsonl 2> $O/gpunode_gpu.err
timeout -k 10 200 $S > $O/unbound_gpu.jsonl 2> $O/unbound_gpu.err
