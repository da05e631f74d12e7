set -e
# Staged-call speed vs CPU / memory placement on one box: copy probe (NUMA
# nodes of CPU, rows, staging, GPU), then the staged call unbound, bound to the
# GPU's NUMA node and bound to the other node (taskset before any GPU use).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06w
mkdir -p $O
cd $R
timeout -k 10 120 $R/tools/host_copy_probe 100 > $O/copy_probe.jsonl 2> $O/copy_probe.err
GN=$(python3 -c "import json; print(json.loads(open('$O/copy_probe.jsonl').readline())['gpu_node'])")
if [ "$GN" -lt 0 ]; then GN=0; fi
ON=$((1 - GN))
GC=$(cat /sys/devices/system/node/node$GN/cpulist)
OC=$(cat /sys/devices/system/node/node$ON/cpulist)
echo "gpu_node=$GN gpu_cpus=$GC other_cpus=$OC" > $O/placement.txt
V="default:0:0:0:0,pinned:262144:4:0:0:0:1:ROWS=pinned"
timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep_unbound.jsonl 2> $O/sweep_unbound.err
timeout -k 10 200 taskset -c $GC $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep_gpunode.jsonl 2> $O/sweep_gpunode.err
timeout -k 10 200 taskset -c $OC $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep_othernode.jsonl 2> $O/sweep_othernode.err
timeout -k 10 120 taskset -c $GC $R/tools/host_copy_probe 100 > $O/copy_probe_gpunode.jsonl 2> $O/copy_probe_gpunode.err
timeout -k 10 120 taskset -c $OC $R/tools/host_copy_probe 100 > $O/copy_probe_othernode.jsonl 2> $O/copy_probe_othernode.err
