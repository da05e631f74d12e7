# Round 2: host-batch tests + synth GPU test, then the bench line (with the
# e2e config-5 leg, parity SHA, nproc CPU baseline), and the box's CPU facts.
set -o pipefail
mkdir -p gpurun_out/r02b
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; echo "OMP=$OMP_NUM_THREADS"; } > gpurun_out/r02b/cpu.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_host_batch.py tests/test_synth.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r02b/tests.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r02b/bench.jsonl 2> gpurun_out/r02b/bench.err || exit $?
