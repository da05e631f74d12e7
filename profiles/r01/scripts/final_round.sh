# Round-end GPU pass: parity suite, smoke, per-code rates (pipelined and
# plain runtime kernel), the rocprof round profile and the default bench line.
mkdir -p gpurun_out/final3 && rm -rf gpurun_out/prof
timeout -k 10 300 python tools/sweep_apply.py > gpurun_out/final3/sweep.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final3/gpu_tests.log 2>&1 || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final3/smoke.log 2>&1 || exit $?
for v in 0 1; do
  HRS_PIPE=$v timeout -k 10 300 python tools/bench_codes.py >> gpurun_out/final3/codes_p$v.jsonl 2>&1 || exit $?
done
bash tools/profile_round.sh || exit $?
timeout -k 10 300 python bench.py > gpurun_out/final3/bench.jsonl 2>&1 || exit $?
