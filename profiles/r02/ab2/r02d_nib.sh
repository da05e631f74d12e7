# Nibble-indexed, bank-private Z_1024 tables in the fused encode+CRC
# (HRS_FUSED=4) vs the byte tables (3): parity suite under the new variant,
# then interleaved timings (RS(12,4) also at G = 2).
set -o pipefail
O=gpurun_out/nib
mkdir -p $O
HRS_FUSED=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_encode_crc.py > $O/tests_v4.txt 2>&1 || exit $?
for rep in 1 2 3; do
  for v in 3 4; do
    for kp in "10 4" "12 4" "6 3"; do
      set -- $kp
      echo "{\"HRS_FUSED\": $v}" >> $O/ab.jsonl
      HRS_FUSED=$v timeout -k 10 120 python tools/bench_encode_crc.py --k $1 --p $2 --iters 20 >> $O/ab.jsonl 2>$O/err.txt || exit $?
    done
    echo "{\"HRS_FUSED\": $v, \"HRS_FUSED_GROUP\": 2}" >> $O/ab.jsonl
    HRS_FUSED_GROUP=2 HRS_FUSED=$v timeout -k 10 120 python tools/bench_encode_crc.py --k 12 --p 4 --iters 20 >> $O/ab.jsonl 2>$O/err.txt || exit $?
  done
done
