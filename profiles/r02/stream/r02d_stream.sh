# Streaming runtime kernel (each input read once, each output written once,
# up to 32 inputs per launch) vs the chunked register-resident launches
# (HRS_STREAM=0): parity suites, then interleaved encode timings of shapes
# that needed several launches.
set -o pipefail
O=gpurun_out/stream
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_nrs.py tests/test_src.py tests/test_gpu_fuzz.py tests/test_gpu_exhaustive.py \
  tests/test_batch_decode.py tests/test_host_path.py > $O/tests.txt 2>&1 || exit $?
for rep in 1 2; do
  for v in 0 1; do
    echo "{\"HRS_STREAM\": $v}" >> $O/enc.jsonl
    HRS_STREAM=$v timeout -k 10 200 python tools/bench_encode.py --shapes 20,8 10,6 24,4 32,8 16,4 --iters 10 >> $O/enc.jsonl 2>$O/err.txt || exit $?
  done
done
