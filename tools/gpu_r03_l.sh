#!/bin/bash
# Round 3 (l): pipelined passes (overlap) -- parity (build, C2, C3, multirank), then C3 A/B.
set -u
O=gpurun_out; mkdir -p $O
export GPU_MAX_HW_QUEUES=8
timeout -k 10 900 python3 -u -m pytest -x -q --durations=5 --timeout 400 --timeout-method thread \
  tests/test_gpu_build.py "tests/test_gpu_scale.py::test_c2_build_bit_exact" tests/test_gpu_c3.py tests/test_gpu_multirank.py \
  > $O/r03_l.log 2>&1; rc=$?
tail -4 $O/r03_l.log
[ $rc -ne 0 ] && exit $rc
bash tools/c3_opts.sh "" "overlap=0" "serial_overflow=1" "side_cus=128"
