# A/B record: a pipelined XOR kernel (HRS_PIPE_XOR) measured neutral (no math to overlap) and was removed; output in profiles/r01/pipe/xor_ab.
OUT=gpurun_out/xorab
mkdir -p $OUT
HRS_PIPE_XOR=1 timeout -k 10 300 python -u -m pytest tests/test_xor.py -x -q --timeout 120 --timeout-method thread > $OUT/xor_tests_pipe.log 2>&1 || exit $?
for run in 1 2 3; do
  for v in 0 1; do
    HRS_PIPE_XOR=$v timeout -k 10 300 python tools/bench_codes.py >> $OUT/codes_x$v.jsonl 2>&1 || exit $?
  done
done
