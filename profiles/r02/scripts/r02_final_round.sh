# Round-2 (final session) GPU pass on the current tree: -m gpu suite, smoke,
# the default bench line, then the rocprof kernel trace + FETCH/WRITE/SQ
# counter passes of the same bench command (profiles/run_rocprof.sh).
set -o pipefail
O=gpurun_out/r02d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.jsonl 2> $O/bench_err.txt || exit $?
bash profiles/run_rocprof.sh $O/prof --no-e2e --no-sha || exit $?
