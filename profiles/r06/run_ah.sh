set -e
# The pageable host-batch gap between bench.py's e2e leg and bench_hbatch.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ah
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/pageable_gap_probe.py > $O/probe.jsonl 2> $O/probe.err
timeout -k 10 300 python -u tools/pageable_gap_probe.py >> $O/probe.jsonl 2>> $O/probe.err
