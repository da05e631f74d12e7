set -o pipefail
mkdir -p gpurun_out/fused2
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 60 rocprofv3 -L > gpurun_out/fused2/counters.txt 2>&1 || true
for v in "3 1" "3 2" "1 1"; do
  set -- $v
  HRS_FUSED=$1 HRS_FUSED_RING=$2 timeout -k 10 300 python -u -m pytest tests/test_encode_crc.py -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/fused2/tests_v$1_r$2.txt 2>&1 || exit $?
  for kp in "10 4" "12 4"; do
    set -- $v $kp
    HRS_FUSED=$1 HRS_FUSED_RING=$2 timeout -k 10 120 python tools/bench_encode_crc.py --k $3 --p $4 \
      | sed "s/^{/{\"variant\": \"v$1 ring $2\", /" >> gpurun_out/fused2/ab.jsonl || exit $?
  done
done
HRS_FUSED=3 HRS_FUSED_RING=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d gpurun_out/fused2/pmc1 -o run -- python tools/bench_encode_crc.py --iters 2 > gpurun_out/fused2/pmc1.txt 2>&1 || exit $?
timeout -k 10 120 tools/copy_probe > gpurun_out/fused2/copy_probe.json 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/fused2/copy_trace -o run -- tools/copy_probe > gpurun_out/fused2/copy_trace.txt 2>&1 || exit $?
