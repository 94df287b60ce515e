#!/bin/bash
# Round 3 (o): the heavy-key sort in rounds of 4 items per thread -- parity (build incl. the
# heavy-split tests, C2, C3), then C3.
set -u
O=gpurun_out; mkdir -p $O
export GPU_MAX_HW_QUEUES=8
timeout -k 10 900 python3 -u -m pytest -x -q --durations=5 --timeout 400 --timeout-method thread \
  tests/test_gpu_build.py "tests/test_gpu_scale.py::test_c2_build_bit_exact" tests/test_gpu_c3.py \
  > $O/r03_o.log 2>&1; rc=$?
tail -4 $O/r03_o.log
[ $rc -ne 0 ] && exit $rc
bash tools/c3_opts.sh "" ""
