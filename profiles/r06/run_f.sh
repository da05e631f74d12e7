set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06f
mkdir -p $O
V="c256_s4:262144:4:0:0,c512_s2:524288:2:0:0,q64:65536:1:0:2,q128:131072:1:0:2,q256:262144:1:0:2,q32:32768:1:0:2"
HRS_HOST_PIECE=262144 timeout -k 10 200 $R/tools/host_pipeline_sweep 100 5 1048576 "$V" > $O/sweep.jsonl 2> $O/sweep.err
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_host_path.py tests/test_host_crc.py tests/test_host_memory.py > $O/tests.txt 2>&1
