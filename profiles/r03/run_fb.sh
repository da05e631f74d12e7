#!/bin/bash
# Round-3 final profile of the tree with the fused repair + CRC: its suite
# (incl. the mirror's device-row checksum methods), then rocprofv3 kernel
# trace + FETCH / WRITE / SQ passes of the default bench.
set -e
mkdir -p gpurun_out/r03fb
timeout -k 10 300 python -u -m pytest tests/test_decode_crc.py tests/test_host_crc.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03fb/decode_crc_tests.txt 2>&1
bash profiles/run_rocprof.sh gpurun_out/r03fb
