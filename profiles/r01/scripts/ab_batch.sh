# A/B record: the pipelined batch kernel (HRS_PIPE_BATCH) measured neutral and was removed; this script produced profiles/r01/pipe/batch_ab_patv.
OUT=gpurun_out/batchab3
mkdir -p $OUT
HRS_PIPE_BATCH=1 timeout -k 10 300 python -u -m pytest tests/test_batch_decode.py tests/test_gpu_exhaustive.py -x -q --timeout 120 --timeout-method thread > $OUT/batch_tests_pipe.log 2>&1 || exit $?
for run in 1 2 3; do
  for v in 0 1; do
    HRS_PIPE_BATCH=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 >> $OUT/bench_b$v.jsonl 2>&1 || exit $?
  done
done
