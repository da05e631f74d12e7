set -e
# Pageable host batches on one box: bench_hbatch (merged vs separate copy
# batches) and bench.py's e2e_config5 leg with each, plus the copy probe.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06af
mkdir -p $O
cd $R
timeout -k 10 120 $R/tools/host_copy_probe 20 > $O/copy_probe.jsonl 2> $O/copy_probe.err
timeout -k 10 400 python -u tools/bench_hbatch.py --reps 3 --zc-blocks > $O/hbatch.jsonl 2> $O/hbatch.err
timeout -k 10 400 python bench.py --no-cpu-baseline --no-host-calls > $O/bench_merge.jsonl 2> $O/bench_merge.err
HRS_HBATCH_MERGE=0 timeout -k 10 400 python bench.py --no-cpu-baseline --no-host-calls > $O/bench_nomerge.jsonl 2> $O/bench_nomerge.err
