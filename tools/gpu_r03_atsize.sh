#!/bin/bash
# Round 3: the at-size parity tests (C3 slice + properties, C4 10M, C5 100K) and the redo canary.
set -u
O=gpurun_out; mkdir -p $O
export GPU_MAX_HW_QUEUES=8
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread \
  "tests/test_gpu_build.py::test_work_buffers_grow_and_redo" \
  tests/test_gpu_c3.py tests/test_gpu_scale.py "tests/test_gpu_matrix.py::test_c5_full_100k_bit_exact" \
  > $O/r03_atsize.log 2>&1; rc=$?
tail -25 $O/r03_atsize.log; exit $rc
