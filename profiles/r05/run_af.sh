#!/bin/bash
# Round 5: the middle launched before the head / tail staging copies.
# Host-path GPU suites under all three transfer modes, the
# C-ABI call rate direct vs staged (interleaved, 3 passes), then the bench.
O=gpurun_out/r05af
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_host_direct.py \
  tests/test_host_path.py tests/test_host_crc.py tests/test_jni.py tests/test_cpp_harness.py > $O/tests.txt 2>&1
rc=$?
if [ $rc -gt 1 ]; then exit $rc; fi
for rep in 1 2 3; do
  for d in 1 0; do
    HRS_HOST_DIRECT=$d timeout -k 10 60 ./tools/host_call_rate 300 > $O/rate_d${d}_r$rep.jsonl 2> $O/rate_d${d}_r$rep.err || exit $?
  done
done
timeout -k 10 500 python bench.py --no-cpu-baseline > $O/bench.jsonl 2> $O/bench.err
