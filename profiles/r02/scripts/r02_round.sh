# Round-2 GPU pass: -m gpu suite, smoke, the default bench line, the rocprof
# kernel trace + separate FETCH_SIZE / WRITE_SIZE passes of the same bench
# command (profiles/run_rocprof.sh), the fused encode+CRC A/B with its
# counters, the concurrent-handle rates and the copy probe.
set -o pipefail
O=gpurun_out/r02
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.jsonl 2> $O/bench_err.txt || exit $?
bash profiles/run_rocprof.sh $O/prof --no-e2e --no-sha || exit $?
for v in "1 2" "2 2" "2 1" "2 4"; do
  set -- $v
  HRS_FUSED=$1 HRS_FUSED_GROUP=$2 timeout -k 10 120 python tools/bench_encode_crc.py \
    | sed "s/^{/{\"variant\": \"form$1 group$2\", /" >> $O/fused_ab.jsonl || exit $?
done
for t in 1 2 4 8; do
  timeout -k 10 120 tests/cpp/codec_harness --threads=$t --rounds=40 10 4 1048576 1048576 1 31 >> $O/threads.jsonl 2>&1 || exit $?
done
timeout -k 10 120 tools/copy_probe > $O/copy_probe.json 2>&1 || exit $?
