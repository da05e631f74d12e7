# Round 2, first GPU pass: the whole -m gpu suite (new: JNI fake-env, SRC at
# compiled shapes, config-1 fixture, Decoder restart, concurrent handles),
# then the concurrent-handle rates at 1/2/4/8 threads.
set -o pipefail
mkdir -p gpurun_out/r02a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r02a/gpu_tests.log 2>&1 || exit $?
for t in 1 2 4 8; do
  timeout -k 10 120 tests/cpp/codec_harness --threads=$t --rounds=40 10 4 1048576 1048576 1 31 \
    >> gpurun_out/r02a/threads.jsonl 2>&1 || exit $?
done
