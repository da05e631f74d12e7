# A/B of the batch kernel's pattern-index prefetch (HRS_BATCH_PATV=0/1), three alternating bench runs each.
OUT=gpurun_out/batchab2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_batch_decode.py -x -q --timeout 120 --timeout-method thread > $OUT/batch_tests.log 2>&1 || exit $?
for run in 1 2 3; do
  for v in 0 1; do
    HRS_BATCH_PATV=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 >> $OUT/bench_v$v.jsonl 2>&1 || exit $?
  done
done
