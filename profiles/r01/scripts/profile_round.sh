# Round profile: bench trace + stats and separate FETCH/WRITE PMC passes
# (profiles/run_rocprof.sh), then a kernel trace of the per-code rates.
set -e
OUT=gpurun_out/prof
bash profiles/run_rocprof.sh $OUT
REPO=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/$OUT/codes_trace" -o run -- \
  python3 "$REPO/tools/bench_codes.py" --iters 5 > "$REPO/$OUT/codes_trace.log" 2>&1
