set -e
# Narrow (256-thread) fused encode + CRC blocks for zero-copy chunks, A/B in
# one process, and the zero-copy grid cap; then the host-path suites.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06n
mkdir -p $O
cd $R
V="narrow:262144:4:0:0:0:1:HRS_FUSED_NARROW=1,wide:262144:4:0:0:0:1:HRS_FUSED_NARROW=0,narrow_zc128:262144:4:0:0:0:1:HRS_ZC_BLOCKS=128,narrow_zc32:262144:4:0:0:0:1:HRS_ZC_BLOCKS=32,wide_zc128:262144:4:0:0:0:1:HRS_FUSED_NARROW=0+HRS_ZC_BLOCKS=128"
timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep.jsonl 2> $O/sweep.err
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_host_path.py tests/test_host_crc.py tests/test_host_memory.py tests/test_encode_crc.py > $O/tests.txt 2>&1
