set -e
# Final-code long fuzz (unbound), and the pageable batch probe with 0 / 16 GiB
# of device memory held (bench.py holds its 14 GiB workload).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ak
mkdir -p $O
cd $R
timeout -k 10 300 python -u tests/tools/fuzz_long.py 4 1000 > $O/fuzz.jsonl 2> $O/fuzz.err
timeout -k 10 300 python -u tools/pageable_gap_probe.py > $O/probe.jsonl 2> $O/probe.err
PROBE_HOLD_GIB=16 timeout -k 10 300 python -u tools/pageable_gap_probe.py >> $O/probe.jsonl 2>> $O/probe.err
PROBE_HOLD_GIB=64 timeout -k 10 300 python -u tools/pageable_gap_probe.py >> $O/probe.jsonl 2>> $O/probe.err
