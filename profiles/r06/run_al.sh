set -e
# bench.py's pageable config-5 leg: which earlier part of the bench process
# slows it (35 ms vs 30 ms in a fresh process)? Default, --no-sha, --stripes 64.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06al
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py --no-cpu-baseline --no-host-calls > $O/default.jsonl 2> $O/default.err
timeout -k 10 400 python bench.py --no-cpu-baseline --no-host-calls --no-sha > $O/nosha.jsonl 2> $O/nosha.err
timeout -k 10 400 python bench.py --no-cpu-baseline --no-host-calls --stripes 64 > $O/s64.jsonl 2> $O/s64.err
