#!/bin/bash
# Round 5: the direct path's rare corruption vs transparent huge pages
# (numpy madvises large arrays MADV_HUGEPAGE; khugepaged may then collapse
# registered, unpinned pages): the long fuzz sequence by default, with numpy's
# THP advice off, and by default again.
O=gpurun_out/r05at
mkdir -p $O
timeout -k 10 400 python -u tests/tools/fuzz_long.py 6 2000 > $O/default_1.jsonl 2> $O/default_1.err
timeout -k 10 400 python -u tests/tools/fuzz_long.py 6 2000 --no-thp > $O/nothp_1.jsonl 2> $O/nothp_1.err
timeout -k 10 400 python -u tests/tools/fuzz_long.py 6 2000 --no-thp > $O/nothp_2.jsonl 2> $O/nothp_2.err
grep -E "thp|AnonHugePages" /proc/meminfo > $O/meminfo.txt; cat /sys/kernel/mm/transparent_hugepage/khugepaged/pages_collapsed >> $O/meminfo.txt 2>&1
