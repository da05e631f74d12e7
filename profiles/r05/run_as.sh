#!/bin/bash
# Round 5: is the direct path's rare corruption the kernel's NUMA balancing
# moving registered (not pinned) pages? The long fuzz sequence twice with an
# explicit MPOL_LOCAL policy (NUMA balancing skips such pages), after
# recording the box's NUMA settings.
O=gpurun_out/r05as
mkdir -p $O
{ cat /proc/sys/kernel/numa_balancing; ls /sys/devices/system/node/ | grep -c node; cat /sys/kernel/mm/transparent_hugepage/enabled; \
  cat /proc/sys/vm/compact_unevictable_allowed 2>/dev/null; uname -r; } > $O/sys.txt 2>&1
for rep in 1 2; do
  timeout -k 10 500 python -u tests/tools/fuzz_long.py 6 2000 --local-mempolicy > $O/local_$rep.jsonl 2> $O/local_$rep.err || exit $?
done
