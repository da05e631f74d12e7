#!/bin/bash
# Round 5, first box: the gfx950 counter list (for the SQC instruction-cache
# pass of the fused encode + CRC kernel) and a baseline of that kernel.
set -e
O=gpurun_out/r05a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -k 10 200 python tools/bench_encode_crc.py --iters 10 > $O/encode_crc.jsonl 2> $O/encode_crc.err
