#!/bin/bash
# Round 3 (i): fewer barriers per group-by batch (one-barrier scans, merged class count) --
# parity (build, C2, C3), stamps, C3 A/B incl. flag_check.
set -u
O=gpurun_out; mkdir -p $O
export GPU_MAX_HW_QUEUES=8
timeout -k 10 900 python3 -u -m pytest -x -q --durations=5 --timeout 400 --timeout-method thread \
  tests/test_gpu_build.py "tests/test_gpu_scale.py::test_c2_build_bit_exact" tests/test_gpu_c3.py \
  > $O/r03_i.log 2>&1; rc=$?
tail -4 $O/r03_i.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/diag_build.py --steps 1 > $O/r03_diag_i.log 2>&1; rc=$?
grep -A 14 "^stamps" $O/r03_diag_i.log; grep "^timings" $O/r03_diag_i.log | tail -1
[ $rc -ne 0 ] && exit $rc
bash tools/c3_opts.sh "" "flag_check=1" ""
