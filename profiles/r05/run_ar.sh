#!/bin/bash
# Round 5: the long fuzz sequence that failed once (tests/tools/fuzz_long.py
# 6 2000), direct path (default) then staged (HRS_HOST_DIRECT=0).
O=gpurun_out/r05ar
mkdir -p $O
timeout -k 10 500 python -u tests/tools/fuzz_long.py 6 2000 > $O/direct.jsonl 2> $O/direct.err
HRS_HOST_DIRECT=0 timeout -k 10 500 python -u tests/tools/fuzz_long.py 6 2000 > $O/staged.jsonl 2> $O/staged.err
