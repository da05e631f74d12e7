#!/bin/bash
# Round 5: concurrent asynchronous codecs (bench.py's async_rounds leg failed
# its check on the first box), staged vs page-registered synchronous calls,
# and the sync-call slot x chunk sweep.
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_async_threads.py \
  tests/test_async.py > $O/async_tests.txt 2>&1
rc=$?
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 ./tools/register_zc_probe 100 > $O/register_probe.jsonl 2> $O/register_probe.err || exit $?
bash profiles/r05/run_f.sh
