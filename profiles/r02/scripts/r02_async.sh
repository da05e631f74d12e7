# Async-round tests + timing, then the fused-kernel LDS counters.
set -o pipefail
O=gpurun_out/async
mkdir -p $O
timeout -k 10 120 ./tests/cpp/codec_harness --async=2 10 4 16781313 1048576 2 17 > $O/diag.json 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_async.py \
  tests/test_jni.py "tests/test_cpp_harness.py::test_harness_async_rounds_vs_sync" > $O/tests.txt 2>&1 || exit $?
for d in 1 2 3 4; do
  timeout -k 10 120 ./tests/cpp/codec_harness --async=$d 10 4 67108864 1048576 2 5 >> $O/async.jsonl 2>&1 || exit $?
done
timeout -k 10 120 ./tests/cpp/codec_harness --async=3 10 4 67108864 4194304 2 5 >> $O/async.jsonl 2>&1 || exit $?
timeout -k 10 120 ./tests/cpp/codec_harness --async=3 12 4 67108864 1048576 4 5 >> $O/async.jsonl 2>&1 || exit $?
bash tools/r02_fused_pmc.sh
