# Decode with two windows per wave task (HRS_DEC_W2=1: 4 KiB contiguous
# stores) vs the pipelined product kernel, 1-2 erasures; parity suite first.
set -o pipefail
O=gpurun_out/w2
mkdir -p $O
HRS_DEC_W2=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_nrs.py > $O/tests_w2.txt 2>&1 || exit $?
for rep in 1 2 3; do
  for v in 0 1; do
    echo "{\"HRS_DEC_W2\": $v}" >> $O/codes.jsonl
    HRS_DEC_W2=$v timeout -k 10 200 python tools/bench_codes.py --iters 10 >> $O/codes.jsonl 2>$O/err.txt || exit $?
  done
done
