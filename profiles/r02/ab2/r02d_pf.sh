# Prefetching fused encode+CRC (HRS_FUSED=4: 768 threads, 5: 1024, 6: 512)
# vs the grouped default (3): parity suites under each new variant, then
# interleaved timings at RS(10,4) / RS(12,4) / RS(6,3).
set -o pipefail
O=gpurun_out/pf
mkdir -p $O
for v in 4 6; do
  HRS_FUSED=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_encode_crc.py > $O/tests_v$v.txt 2>&1 || exit $?
done
for rep in 1 2; do
  for v in 3 4 6 5; do
    for kp in "10 4" "12 4" "6 3"; do
      set -- $kp
      echo "{\"HRS_FUSED\": $v}" >> $O/ab.jsonl
      HRS_FUSED=$v timeout -k 10 120 python tools/bench_encode_crc.py --k $1 --p $2 --iters 20 >> $O/ab.jsonl 2>$O/err.txt || exit $?
    done
  done
done
