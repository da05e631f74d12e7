# Factored XOR network in the fused encode+CRC (now the default): the GPU
# suites that reach the fused kernel, then interleaved A/B timings of the
# default vs the paired network (HRS_FUSED=2) at RS(10,4) and RS(12,4).
# (Round-2 first pass of this script also A/B'd the factored network in the
# plain encode kernel: slower at every shape, profiles/r02/sched/enc_ab.jsonl.)
set -o pipefail
O=gpurun_out/sched2
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_encode_crc.py tests/test_host_crc.py tests/test_src.py tests/test_nrs.py tests/test_async.py > $O/tests.txt 2>&1 || exit $?
for rep in 1 2 3; do
  for v in 3 2; do
    for kp in "10 4" "12 4" "6 3"; do
      set -- $kp
      echo "{\"HRS_FUSED\": $v}" >> $O/ab.jsonl
      HRS_FUSED=$v timeout -k 10 120 python tools/bench_encode_crc.py --k $1 --p $2 --iters 20 >> $O/ab.jsonl 2>/dev/null || exit $?
    done
  done
done
