#!/bin/bash
# Round 4 final pass on the final tree: copy pool + host-call rates, the full
# GPU suite, smoke, the default bench, then the rocprofv3 kernel trace and the
# FETCH / WRITE / SQ counter passes of the bench (profiles/run_rocprof.sh).
set -e
O=gpurun_out/r04k
mkdir -p $O
for t in 0 2 4 8 15; do
  HRS_HOST_THREADS=$t timeout -k 10 60 ./tools/pool_probe > $O/pool_t$t.jsonl 2> $O/pool_t$t.err
done
timeout -k 10 120 python tools/bench_host_api.py --calls 40 > $O/host_api.jsonl 2> $O/host_api.err
timeout -k 10 120 python tools/bench_host_ab.py --calls 40 > $O/host_ab.jsonl 2> $O/host_ab.err
timeout -k 10 120 ./tests/cpp/codec_harness --threads=1 --rounds=64 10 4 > $O/harness_t1.jsonl 2> $O/harness_t1.err
timeout -k 10 120 ./tests/cpp/codec_harness --threads=4 --rounds=32 10 4 > $O/harness_t4.jsonl 2> $O/harness_t4.err
timeout -k 10 300 python tools/bench_hbatch.py --reps 3 --zc-blocks > $O/hbatch_ab.jsonl 2> $O/hbatch_ab.err
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 400 python bench.py > $O/bench.jsonl 2> $O/bench.err
bash profiles/run_rocprof.sh $O/prof
