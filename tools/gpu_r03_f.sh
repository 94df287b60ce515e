#!/bin/bash
# Round 3 (f): fused pass selection + coalesced bucket emit + padded stage cursors + half-round
# stage variant -- parity (build, C2, C3, CLI), stamps, short C3 bench, stage_round A/B.
set -u
O=gpurun_out; mkdir -p $O
export GPU_MAX_HW_QUEUES=8
timeout -k 10 900 python3 -u -m pytest -x -q --durations=5 --timeout 400 --timeout-method thread \
  tests/test_gpu_build.py "tests/test_gpu_scale.py::test_c2_build_bit_exact" tests/test_gpu_c3.py tests/test_gpu_cli.py \
  > $O/r03_f.log 2>&1; rc=$?
tail -10 $O/r03_f.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/diag_build.py --steps 1 > $O/r03_diag_f.log 2>&1; rc=$?
grep -A 14 "^stamps" $O/r03_diag_f.log; grep "^timings" $O/r03_diag_f.log | tail -1
[ $rc -ne 0 ] && exit $rc
bash tools/c3_opts.sh "" "stage_round=1"
