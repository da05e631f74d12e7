set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06j
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py > $O/bench.jsonl 2> $O/bench.err
timeout -k 10 400 bash profiles/run_rocprof.sh $O/prof > $O/prof.log 2>&1
