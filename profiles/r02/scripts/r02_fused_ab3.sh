set -o pipefail
mkdir -p gpurun_out/fused3
for g in 2 4; do
  HRS_FUSED=4 HRS_FUSED_GROUP=$g timeout -k 10 300 python -u -m pytest tests/test_encode_crc.py -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/fused3/tests_g$g.txt 2>&1 || exit $?
done
for v in "3 1" "4 1" "4 2" "4 3" "4 4"; do
  set -- $v
  for kp in "10 4" "12 4" "6 3"; do
    set -- $v $kp
    HRS_FUSED=$1 HRS_FUSED_RING=1 HRS_FUSED_GROUP=$2 timeout -k 10 120 python tools/bench_encode_crc.py --k $3 --p $4 \
      | sed "s/^{/{\"variant\": \"v$1 g$2\", /" >> gpurun_out/fused3/ab.jsonl || exit $?
  done
done
