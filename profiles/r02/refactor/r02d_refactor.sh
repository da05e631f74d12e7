# accumulate_row refactor: same-box A/B against the previous build (HRS_LIB)
# on the runtime and batch kernels, after the suites that reach them.
set -o pipefail
O=gpurun_out/refactor
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_batch_decode.py tests/test_gpu_fuzz.py tests/test_src.py tests/test_nrs.py > $O/tests.txt 2>&1 || exit $?
for rep in 1 2; do
  for lib in ablib/libhrs_prev.so lambdafs_amd/libhrs.so; do
    echo "{\"lib\": \"$lib\"}" >> $O/codes.jsonl
    HRS_LIB=$PWD/$lib timeout -k 10 200 python tools/bench_codes.py --iters 10 >> $O/codes.jsonl 2>$O/err.txt || exit $?
    echo "{\"lib\": \"$lib\"}" >> $O/batch.jsonl
    HRS_LIB=$PWD/$lib timeout -k 10 120 python tools/bench_batch_wide.py --k 10 --p 4 --stripes 1024 --cell 1048576 >> $O/batch.jsonl 2>>$O/err.txt || exit $?
  done
done
