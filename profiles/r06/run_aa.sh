set -e
# Long seeded fuzz and fresh-buffer reuse on the final staged defaults
# (nontemporal copy-ins, spinning pool on the GPU's node), unbound and from
# the other socket.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06aa
mkdir -p $O
cd $R
timeout -k 10 300 python -u tests/tools/fuzz_long.py 6 1000 > $O/fuzz_unbound.jsonl 2> $O/fuzz_unbound.err
GN=$(cat /sys/bus/pci/devices/$(python3 -c "print('x')" >/dev/null; ls /sys/bus/pci/drivers/amdgpu 2>/dev/null | grep -m1 ':' )/numa_node 2>/dev/null || echo 0)
if [ "$GN" -lt 0 ] 2>/dev/null; then GN=0; fi
ON=$((1 - GN))
OC=$(cat /sys/devices/system/node/node$ON/cpulist)
echo "gpu_node(guess)=$GN other_cpus=$OC" > $O/placement.txt
timeout -k 10 300 taskset -c $OC python -u tests/tools/fuzz_long.py 4 1000 > $O/fuzz_other.jsonl 2> $O/fuzz_other.err
timeout -k 10 300 python -u tests/tools/fresh_buffer_repro.py 400 > $O/reuse.txt 2> $O/reuse.err
