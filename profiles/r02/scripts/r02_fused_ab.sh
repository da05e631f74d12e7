# Fused encode + CRC: correctness of every variant, then rates (same process
# per variant, RS(10,4) and RS(12,4), 1,024 x 1 MiB stripes).
set -o pipefail
mkdir -p gpurun_out/fused
for v in "3 2" "3 1" "1 1"; do
  set -- $v
  HRS_FUSED=$1 HRS_FUSED_RING=$2 timeout -k 10 300 python -u -m pytest tests/test_encode_crc.py -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/fused/tests_v$1_r$2.log 2>&1 || exit $?
done
for v in "1 1" "3 1" "3 2" "3 3" "3 4"; do
  set -- $v
  for kp in "10 4" "12 4" "6 3"; do
    set -- $v $kp
    HRS_FUSED=$1 HRS_FUSED_RING=$2 timeout -k 10 120 python tools/bench_encode_crc.py --k $3 --p $4 \
      | sed "s/^{/{\"variant\": \"v$1 ring $2\", /" >> gpurun_out/fused/ab.jsonl || exit $?
  done
done
