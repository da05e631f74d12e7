#!/bin/bash
# rocprofv3 recipe for the bench workload (run on the GPU box from the repo root):
#   1. kernel trace + stats           -> per-kernel average duration
#   2. --pmc FETCH_SIZE (own pass)    -> HBM read KiB per dispatch (gfx950: x2 for wide streams)
#   3. --pmc WRITE_SIZE (own pass)    -> HBM write KiB per dispatch
#   4. --pmc SQ_* (own pass)          -> wave-cycle split (busy / parked / issue-stalled, VALU, LDS)
# Usage: bash profiles/run_rocprof.sh <outdir> [bench args...]
set -e
OUT=$(realpath -m "$1"); shift
REPO=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$REPO/bench.py" --no-cpu-baseline --no-host-calls "$@" > "$OUT/trace_bench.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
  python3 "$REPO/bench.py" --no-cpu-baseline --no-host-calls "$@" > "$OUT/pmc_fetch_bench.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
  python3 "$REPO/bench.py" --no-cpu-baseline --no-host-calls "$@" > "$OUT/pmc_write_bench.log" 2>&1
cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d "$OUT/pmc_sq" -o run -- \
  python3 "$REPO/bench.py" --no-cpu-baseline --no-host-calls "$@" > "$OUT/pmc_sq_bench.log" 2>&1
