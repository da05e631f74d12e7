set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06l
mkdir -p $O
cd $R
V="c256_s4:262144:4:0:0:0:1,c256_s4_gpufold:262144:4:0:0:0:0,c512_s2:524288:2:0:0:0:1,c512_s2_gpufold:524288:2:0:0:0:0,c128_s4:131072:4:0:0:0:1,c256_s3:262144:3:0:0:0:1"
timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep.jsonl 2> $O/sweep.err
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_host_path.py tests/test_host_crc.py tests/test_host_memory.py tests/test_encode_crc.py tests/test_decode_crc.py > $O/tests.txt 2>&1
