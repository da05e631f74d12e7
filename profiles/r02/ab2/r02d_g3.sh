# Fused encode+CRC rows per lockstep group G = 2 / 3 / 4 (HRS_FUSED_GROUP),
# factored networks with the new G = 3 schedules: parity suite at G = 3, then
# interleaved timings at RS(10,4), RS(12,4), RS(6,3).
set -o pipefail
O=gpurun_out/g3
mkdir -p $O
HRS_FUSED_GROUP=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_encode_crc.py tests/test_host_crc.py > $O/tests_g3.txt 2>&1 || exit $?
for rep in 1 2 3; do
  for g in 2 3 4; do
    for kp in "10 4" "12 4" "6 3"; do
      set -- $kp
      echo "{\"HRS_FUSED_GROUP\": $g}" >> $O/ab.jsonl
      HRS_FUSED_GROUP=$g timeout -k 10 120 python tools/bench_encode_crc.py --k $1 --p $2 --iters 20 >> $O/ab.jsonl 2>$O/err.txt || exit $?
    done
  done
done
