#!/bin/bash
# Round 4, first GPU pass (measurement only, no product change yet):
#  1. copy schedule lab: which 1:1 copy reaches the guide's 6.29 TB/s here;
#  2. duplex probe: is pinned H2D + D2H concurrent faster than serial;
#  3. synchronous host-buffer call rate vs copy threads / chunk size.
set -e
O=gpurun_out/r04a
mkdir -p $O/host
nproc > $O/nproc.txt; cat /sys/fs/cgroup/cpu.max >> $O/nproc.txt 2>/dev/null || true
timeout -k 10 240 ./tools/copy_lab 7 4 > $O/copy_lab.jsonl 2> $O/copy_lab.err
timeout -k 10 240 python tools/duplex_probe.py --reps 5 > $O/duplex.json 2> $O/duplex.err
for t in 2 4 8 12 16; do
  for ch in 262144 524288 1048576; do
    HRS_HOST_THREADS=$t HRS_HOST_CHUNK=$ch timeout -k 10 120 python tools/bench_host_api.py --calls 40 > $O/host/t${t}_c${ch}.json 2>&1
  done
done
