# Copy-pool threads (HRS_HOST_THREADS) vs the host-memory batch legs of the
# bench (config 5 e2e, pinned and pageable) and the single-stripe sync calls.
set -o pipefail
O=gpurun_out/hthreads
mkdir -p $O
for rep in 1 2; do
  for t in 2 4 8; do
    echo "{\"HRS_HOST_THREADS\": $t}" >> $O/e2e.jsonl
    HRS_HOST_THREADS=$t timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-sha --steps 3 --warmup 1 >> $O/e2e.jsonl 2>$O/err.txt || exit $?
    echo "{\"HRS_HOST_THREADS\": $t}" >> $O/host.jsonl
    HRS_HOST_THREADS=$t timeout -k 10 120 python tools/bench_host_api.py >> $O/host.jsonl 2>>$O/err.txt || exit $?
  done
done
