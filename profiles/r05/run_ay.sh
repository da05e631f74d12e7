#!/bin/bash
# Round 5: staged synchronous calls with the chunk kernels in order on one
# stream and finished chunks copied out early, vs a stream per slot
# (HRS_HOST_ONE_STREAM=0), over chunk size x slots; host-path suites first.
O=gpurun_out/r05ay
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_host_path.py \
  tests/test_host_crc.py tests/test_host_direct.py tests/test_jni.py tests/test_cpp_harness.py > $O/tests.txt 2>&1 || exit $?
for rep in 1 2; do
  for one in 1 0; do
    for ch in 262144 524288; do
      for sl in 2 4; do
        HRS_HOST_ONE_STREAM=$one HRS_HOST_CHUNK=$ch HRS_HOST_SLOTS=$sl timeout -k 10 60 ./tools/host_call_rate 300 \
          | sed "s/^{/{\"one\": $one, \"chunk\": $ch, \"slots\": $sl, \"rep\": $rep, /" >> $O/sweep.jsonl || exit $?
      done
    done
  done
done
