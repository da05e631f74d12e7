#!/bin/bash
# Round 5: the new device-set, scalar-decode and JNI tests on the GPU.
set -e
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_device_set.py tests/test_jni.py "tests/test_gpu_parity.py::test_scalar_decode5_leaves_unlisted_erased_values" \
  "tests/test_gpu_parity.py::test_scalar_encode_decode_like_TestErasureCodes" > $O/tests.txt 2>&1
