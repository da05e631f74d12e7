# Paired coefficient bits in the runtime-matrix kernels (mul_acc_coeffs):
# parity suites on the new build, then interleaved A/B against the previous
# build (ablib/libhrs_base.so via HRS_LIB): rs/nrs/xor decode 1-4 erasures,
# runtime-kernel encodes (RS(20,8), RS(16,4)).
set -o pipefail
O=gpurun_out/pair
mkdir -p $O
# (suites ran green in the first call) timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
#  tests/test_gpu_parity.py tests/test_batch_decode.py tests/test_pipe_kernel.py tests/test_src.py tests/test_nrs.py \
#  tests/test_gpu_fuzz.py tests/test_gpu_exhaustive.py tests/test_xor.py > $O/tests.txt 2>&1 || exit $?
for rep in 1 2; do
  for lib in ablib/libhrs_base.so lambdafs_amd/libhrs.so; do
    echo "{\"lib\": \"$lib\"}" >> $O/codes.jsonl
    HRS_LIB=$PWD/$lib timeout -k 10 200 python tools/bench_codes.py --iters 10 >> $O/codes.jsonl 2>$O/err.txt || exit $?
    echo "{\"lib\": \"$lib\"}" >> $O/enc.jsonl
    HRS_LIB=$PWD/$lib timeout -k 10 120 python tools/bench_encode.py --shapes 20,8 16,4 --iters 10 >> $O/enc.jsonl 2>>$O/err.txt || exit $?
  done
done
