#!/bin/bash
# parity of the build after a k_bucket_process change: unit / key-range / rank-group tests, the C2
# builds and the C3 slice
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_build.py tests/test_gpu_multirank.py tests/test_gpu_chains.py \
  tests/test_gpu_scale.py::test_c2_build_bit_exact tests/test_gpu_c3.py -m gpu -x -v -s --timeout 400 \
  --timeout-method thread > $O/r04_p_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/r04_p_tests.log
exit $rc
