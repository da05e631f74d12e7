set -e
# Host batches: copy-outs merged with the next copy-in (always), ordered
# zero-copy chunks and chunk sizes (A/B); suites first. Then smaller first
# chunks of the synchronous staged call.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ad
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_host_batch.py tests/test_device_set.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1
timeout -k 10 400 python -u tools/bench_hbatch.py --reps 3 --zc-blocks > $O/hbatch.jsonl 2> $O/hbatch.err
V="default:0:0:0:0:1,f64k:131072:8:65536:0:1,f32k:131072:8:32768:0:1,c160_f64k:163840:8:65536:0:1,pinned:0:0:0:0:1:1:ROWS=pinned"
timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep.jsonl 2> $O/sweep.err
