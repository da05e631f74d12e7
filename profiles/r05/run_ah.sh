#!/bin/bash
# Round 5 A/B: the direct path's completion wait, event polling (default) vs
# hipStreamSynchronize (HRS_SPIN_WAIT=0); host-path suites first.
O=gpurun_out/r05ah
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_host_direct.py \
  tests/test_host_crc.py tests/test_host_path.py tests/test_async.py > $O/tests.txt 2>&1 || exit $?
for rep in 1 2 3; do
  for w in 1 0; do
    HRS_SPIN_WAIT=$w timeout -k 10 60 ./tools/host_call_rate 300 > $O/rate_w${w}_r$rep.jsonl 2> $O/rate_w${w}_r$rep.err || exit $?
  done
done
