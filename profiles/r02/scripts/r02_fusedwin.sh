# Fused encode+CRC: window sizes + the contiguous-lane variant.
# tests (default variant, then HRS_FUSED=3), then per-shape timings, then A/B.
set -o pipefail
O=gpurun_out/fusedwin
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_encode_crc.py > $O/tests.txt 2>&1 || exit $?
HRS_FUSED=3 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_encode_crc.py > $O/tests_v3.txt 2>&1 || exit $?
for shape in "1 524288" "1 1048576" "4 1048576" "16 1048576" "64 262144" "128 1048576" "512 262144"; do
  set -- $shape
  timeout -k 10 120 python tools/bench_encode_crc.py --stripes $1 --cell $2 --iters 20 >> $O/timing.jsonl 2>&1 || exit $?
done
for v in "2 2" "3 2" "3 4" "2 2" "3 2" "3 4"; do
  set -- $v
  echo "{\"HRS_FUSED\": $1, \"HRS_FUSED_GROUP\": $2}" >> $O/ab.jsonl
  HRS_FUSED=$1 HRS_FUSED_GROUP=$2 timeout -k 10 120 python tools/bench_encode_crc.py --iters 20 >> $O/ab.jsonl 2>&1 || exit $?
done
HRS_FUSED=3 timeout -k 10 120 python tools/bench_encode_crc.py --k 12 --p 4 --iters 20 >> $O/ab.jsonl 2>&1 || exit $?
timeout -k 10 120 python tools/bench_encode_crc.py --k 12 --p 4 --iters 20 >> $O/ab.jsonl 2>&1 || exit $?
