# PMC traffic of the streaming runtime kernel (RS(20,8) / RS(10,6) encodes):
# kernel trace + separate FETCH_SIZE / WRITE_SIZE passes of the same command.
set -o pipefail
O=$(realpath -m gpurun_out/stream_pmc)
mkdir -p $O
REPO=$(pwd)
export TMPDIR=/tmp
cd /tmp
CMD="python3 $REPO/tools/bench_encode.py --shapes 20,8 10,6 --iters 3 --bytes 7"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $CMD > $O/trace.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $CMD > $O/fetch.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $CMD > $O/write.log 2>&1 || exit $?
