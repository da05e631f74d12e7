# A/B of the software-pipelined runtime kernel (HRS_PIPE=0/1) on one box.
OUT=gpurun_out/${1:-pipe3}
mkdir -p $OUT
timeout -k 10 300 python tools/sweep_apply.py > $OUT/sweep.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit $?
for run in 1 2; do
  for v in 0 1; do
    HRS_PIPE=$v timeout -k 10 300 python tools/bench_codes.py >> $OUT/codes_p$v.jsonl 2>&1 || exit $?
  done
done
