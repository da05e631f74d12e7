set -e
# Validation with nontemporal staging copy-ins by default: whole GPU suite, smoke, bench.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06z
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 400 python bench.py > $O/bench.jsonl 2> $O/bench.err
