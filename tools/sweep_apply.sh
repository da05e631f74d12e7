# Debug aid: runtime-kernel shape sweep, then the GPU suite and per-code rates
# for the masked (default) and branchy (HRS_RUNTIME_BRANCHY=1) variants.
mkdir -p gpurun_out/sweep
timeout -k 10 300 python tools/sweep_apply.py > gpurun_out/sweep/masked.txt 2>&1 || exit $?
HRS_RUNTIME_BRANCHY=1 timeout -k 10 300 python tools/sweep_apply.py > gpurun_out/sweep/branchy.txt 2>&1 || exit $?
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/sweep/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_codes.py > gpurun_out/sweep/masked.jsonl 2>&1 || exit $?
HRS_RUNTIME_BRANCHY=1 timeout -k 10 300 python tools/bench_codes.py > gpurun_out/sweep/branchy.jsonl 2>&1 || exit $?
