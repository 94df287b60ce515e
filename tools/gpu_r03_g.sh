#!/bin/bash
# Round 3 (g): pipelined pass selection (2 id loads per thread, next tile ahead) + overlapped
# emit reservations -- parity (build, C2, C3), stamps, then C3 A/B: select_tile, stream_priority.
set -u
O=gpurun_out; mkdir -p $O
export GPU_MAX_HW_QUEUES=8
timeout -k 10 900 python3 -u -m pytest -x -q --durations=5 --timeout 400 --timeout-method thread \
  tests/test_gpu_build.py "tests/test_gpu_scale.py::test_c2_build_bit_exact" tests/test_gpu_c3.py \
  > $O/r03_g.log 2>&1; rc=$?
tail -4 $O/r03_g.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/diag_build.py --steps 1 > $O/r03_diag_g.log 2>&1; rc=$?
grep -A 14 "^stamps" $O/r03_diag_g.log; grep "^timings" $O/r03_diag_g.log | tail -1
[ $rc -ne 0 ] && exit $rc
bash tools/c3_opts.sh "" "select_tile=0" "stream_priority=1"
