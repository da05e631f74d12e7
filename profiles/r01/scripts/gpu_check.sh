# GPU suite, per-code rates, host-path sweep and the bench line, each step under its own limit.
mkdir -p gpurun_out/check
timeout -k 10 300 python tools/sweep_apply.py > gpurun_out/check/apply.txt 2>&1 || exit $?
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/check/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_codes.py > gpurun_out/check/codes.jsonl 2>&1 || exit $?
bash tools/host_sweep.sh || exit $?
timeout -k 10 300 python bench.py > gpurun_out/check/bench.jsonl 2>&1 || exit $?
