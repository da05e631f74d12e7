#!/bin/bash
# Round-3 last pass: the fused repair + CRC suites on the final kernel, a
# rocprofv3 kernel trace of the repair + CRC A/B tool (1-3 lost cells), the
# GPU suite, smoke and the default bench.
set -e
O=gpurun_out/r03v11
mkdir -p $O
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_decode_crc.py tests/test_host_crc.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/decode_crc_tests.txt 2>&1
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/dcrc_trace -o run -- python3 $R/tools/bench_decode_crc.py --reps 1 --erased "4;0,5;1,6,11" > $R/$O/dcrc_trace.log 2>&1)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 400 python bench.py > $O/bench.jsonl 2> $O/bench.err
