# Streaming heterogeneous-batch kernel for wide patterns vs the previous
# build's per-stripe fallback (HRS_LIB=ablib/libhrs_prev.so): batch suites,
# then interleaved timings of RS(20,8) / RS(12,6) / RS(30,6) repair batches.
set -o pipefail
O=gpurun_out/bstream
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_batch_decode.py tests/test_host_batch.py tests/test_src.py tests/test_gpu_fuzz.py > $O/tests.txt 2>&1 || exit $?
for rep in 1 2; do
  for lib in ablib/libhrs_prev.so lambdafs_amd/libhrs.so; do
    for kp in "20 8" "12 6" "30 6"; do
      set -- $kp
      echo "{\"lib\": \"$lib\"}" >> $O/ab.jsonl
      HRS_LIB=$PWD/$lib timeout -k 10 120 python tools/bench_batch_wide.py --k $1 --p $2 >> $O/ab.jsonl 2>$O/err.txt || exit $?
    done
  done
done
