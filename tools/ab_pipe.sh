# A/B of the software-pipelined kernels (HRS_PIPE=0/1) on one box, then the
# round profile of the default (pipelined) build.
mkdir -p gpurun_out/pipe2
timeout -k 10 300 python tools/sweep_apply.py > gpurun_out/pipe2/sweep.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe2/gpu_tests.log 2>&1 || exit $?
for run in 1 2; do
  for v in 0 1; do
    HRS_PIPE=$v timeout -k 10 300 python tools/bench_codes.py >> gpurun_out/pipe2/codes_p$v.jsonl 2>&1 || exit $?
  done
done
for v in 0 1; do
  HRS_PIPE=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/pipe2/bench_p$v.jsonl 2>&1 || exit $?
done
bash tools/profile_round.sh || exit $?
timeout -k 10 300 python bench.py > gpurun_out/pipe2/bench_default.jsonl 2>&1 || exit $?
