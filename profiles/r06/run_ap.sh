set -e
# The whole GPU suite with the process on the socket the GPU is not on.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ap
mkdir -p $O
cd $R
timeout -k 10 120 $R/tools/host_copy_probe 5 > $O/copy_probe.jsonl 2> $O/copy_probe.err
GN=$(python3 -c "import json; print(json.loads(open('$O/copy_probe.jsonl').readline())['gpu_node'])")
if [ "$GN" -lt 0 ]; then GN=0; fi
ON=$((1 - GN))
OC=$(cat /sys/devices/system/node/node$ON/cpulist)
echo "gpu_node=$GN other_cpus=$OC" > $O/placement.txt
timeout -k 10 1000 taskset -c $OC python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1
