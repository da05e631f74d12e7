mkdir -p gpurun_out/ab
timeout -k 10 300 python tools/sweep_apply.py > gpurun_out/ab/sweep_horner.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/gpu_tests.log 2>&1 || exit $?
for v in 0 1 0 1; do
  HRS_RUNTIME_HORNER=$v timeout -k 10 300 python tools/bench_codes.py > gpurun_out/ab/codes_h$v.jsonl.tmp 2>&1 || exit $?
  cat gpurun_out/ab/codes_h$v.jsonl.tmp >> gpurun_out/ab/codes_h$v.jsonl
done
for v in 0 1; do
  HRS_RUNTIME_HORNER=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab/bench_h$v.jsonl 2>&1 || exit $?
done
