# Debug aid: per-code rates vs grid size (HRS_BLOCKS_PER_CU) for both runtime variants.
mkdir -p gpurun_out/grid
for v in 0 1; do
  for b in 1 2 3 4; do
    HRS_RUNTIME_BRANCHY=$v HRS_BLOCKS_PER_CU=$b timeout -k 10 300 python tools/bench_codes.py --iters 6 > gpurun_out/grid/v${v}_b${b}.jsonl 2>&1 || exit $?
  done
done
