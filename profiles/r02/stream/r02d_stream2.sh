# HRS_STREAM=2: the streaming kernel for every runtime-matrix launch, vs the
# default (streaming only where the register-resident kernels need several
# launches): rs/nrs decode 1-4 erasures, RS(16,4) / RS(12,4)-runtime encodes.
set -o pipefail
O=gpurun_out/stream2
mkdir -p $O
for rep in 1 2; do
  for v in 1 2; do
    echo "{\"HRS_STREAM\": $v}" >> $O/codes.jsonl
    HRS_STREAM=$v timeout -k 10 200 python tools/bench_codes.py --iters 10 >> $O/codes.jsonl 2>$O/err.txt || exit $?
    echo "{\"HRS_STREAM\": $v}" >> $O/enc.jsonl
    HRS_STREAM=$v timeout -k 10 200 python tools/bench_encode.py --shapes 16,4 8,4 14,2 --iters 10 >> $O/enc.jsonl 2>>$O/err.txt || exit $?
  done
done
