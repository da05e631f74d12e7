set -o pipefail
mkdir -p gpurun_out/fused4
for g in 2 4 1; do
  HRS_FUSED=5 HRS_FUSED_GROUP=$g timeout -k 10 300 python -u -m pytest tests/test_encode_crc.py tests/test_host_crc.py -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/fused4/tests_g$g.txt 2>&1 || exit $?
done
for v in "4 2" "5 1" "5 2" "5 3" "5 4"; do
  set -- $v
  for kp in "10 4" "12 4" "6 3"; do
    set -- $v $kp
    HRS_FUSED=$1 HRS_FUSED_GROUP=$2 timeout -k 10 120 python tools/bench_encode_crc.py --k $3 --p $4 \
      | sed "s/^{/{\"variant\": \"v$1 g$2\", /" >> gpurun_out/fused4/ab.jsonl || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
HRS_FUSED=5 HRS_FUSED_GROUP=2 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/fused4/pmc_fetch -o run -- python tools/bench_encode_crc.py --iters 2 > gpurun_out/fused4/pmc_fetch.txt 2>&1 || exit $?
HRS_FUSED=5 HRS_FUSED_GROUP=2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d gpurun_out/fused4/pmc_sq -o run -- python tools/bench_encode_crc.py --iters 2 > gpurun_out/fused4/pmc_sq.txt 2>&1 || exit $?
